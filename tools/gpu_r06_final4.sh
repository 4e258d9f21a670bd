#!/bin/bash
# Round 6, final session 4: the §8(f) lines (RT, AC, SS) with their PMC
# sessions; the NIF harness with one context and with a replica (two lanes
# on the one GPU); the N = 2 launcher-less rehearsal.
set -o pipefail
O=gpurun_out/r06f4
mkdir -p $O
for c in RT AC SS; do
  lc=$(echo $c | tr A-Z a-z)
  OUT=$O/prof_$c LITE=1 TAG=r06_$c BENCH_ARGS="--config $c" timeout -k 10 500 bash tools/profile_session.sh > $O/prof_$c.log 2>&1 || { tail -5 $O/prof_$c.log; exit 3; }
  cp $O/prof_$c/pmc_summary.json profiles/pmc_$lc.json
  timeout -k 10 400 python -u bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 4; }
  tail -c 300 $O/bench_$c.json
done
timeout -k 10 420 ./tools/bin/nif_harness 3 scale churn load > $O/harness.jsonl 2> $O/harness.err || { tail -20 $O/harness.err; exit 5; }
VMQGB_REPLICAS=1 timeout -k 10 300 ./tools/bin/nif_harness 3 churn > $O/harness_lanes2.jsonl 2> $O/harness_lanes2.err || { tail -20 $O/harness_lanes2.err; exit 6; }
tail -3 $O/harness_lanes2.jsonl
timeout -k 10 300 python -u bench.py --gpus 2 --force-device 0 --dist-backend gloo --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_C_n2.json 2> $O/bench_C_n2.err || { tail -5 $O/bench_C_n2.err; exit 7; }
tail -c 300 $O/bench_C_n2.json
