#!/bin/bash
# Round 6, final session 2: A, R1 (4,096,000), R2 (4,096,000): LITE PMC
# sessions, then the bench lines (which read those PMC summaries).
set -o pipefail
O=gpurun_out/r06f2
mkdir -p $O
for c in A R1 R2; do
  args="--config $c"; [ $c != A ] && args="$args --r-n 4096000"
  lc=$(echo $c | tr A-Z a-z)
  OUT=$O/prof_$c LITE=1 TAG=r06_$c BENCH_ARGS="$args" timeout -k 10 500 bash tools/profile_session.sh > $O/prof_$c.log 2>&1 || { tail -5 $O/prof_$c.log; exit 3; }
  cp $O/prof_$c/pmc_summary.json profiles/pmc_$lc.json
  timeout -k 10 400 python -u bench.py $args > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 4; }
  tail -c 400 $O/bench_$c.json
done
