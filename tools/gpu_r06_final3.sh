#!/bin/bash
# Round 6, final session 3: D and E: LITE PMC sessions, then the bench lines.
set -o pipefail
O=gpurun_out/r06f3
mkdir -p $O
for c in D E; do
  lc=$(echo $c | tr A-Z a-z)
  OUT=$O/prof_$c LITE=1 TAG=r06_$c BENCH_ARGS="--config $c" timeout -k 10 900 bash tools/profile_session.sh > $O/prof_$c.log 2>&1 || { tail -5 $O/prof_$c.log; exit 3; }
  cp $O/prof_$c/pmc_summary.json profiles/pmc_$lc.json
  timeout -k 10 600 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 4; }
  tail -c 400 $O/bench_$c.json
done
