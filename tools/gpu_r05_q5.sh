#!/bin/bash
# Round 5, final session 5: the §8(f) lines (RT, AC, SS) with their PMC
# sessions again, tagged with the final libvmqgpu build id.
set -o pipefail
O=gpurun_out/r05q5
mkdir -p $O
for c in RT AC SS; do
  lc=$(echo $c | tr A-Z a-z)
  OUT=$O/prof_$c LITE=1 TAG=r05_$c BENCH_ARGS="--config $c" timeout -k 10 500 bash tools/profile_session.sh > $O/prof_$c.log 2>&1 || { tail -5 $O/prof_$c.log; exit 3; }
  cp $O/prof_$c/pmc_summary.json profiles/pmc_$lc.json
  timeout -k 10 400 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 4; }
  tail -c 300 $O/bench_$c.json
done
