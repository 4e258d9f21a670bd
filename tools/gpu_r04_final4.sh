#!/bin/bash
# Round 4 final build, call 4: R1 / R2 at the reference suite's 4,096,000,
# config A, the host-half harness, then build-tagged rocprofv3 sessions of
# RT, AC and SS.
set -o pipefail
O=gpurun_out/final4
mkdir -p $O
timeout -k 10 300 python -u bench.py --config R1 --r-n 4096000 > $O/bench_R1.json 2> $O/bench_R1.err &&
timeout -k 10 300 python -u bench.py --config R2 --r-n 4096000 > $O/bench_R2.json 2> $O/bench_R2.err &&
timeout -k 10 200 python -u bench.py --config A > $O/bench_A.json 2> $O/bench_A.err &&
timeout -k 10 300 tools/bin/nif_harness 3 scale churn load > $O/nif_harness.jsonl 2> $O/nif_harness.err &&
for c in RT AC SS; do
  LITE=1 OUT=$O/prof_$c BENCH_ARGS="--config $c" TAG=r04_$c bash tools/profile_session.sh > $O/prof_$c.log 2>&1 || exit 4
done
# config D's line again, now that pmc_d.json is of this build (traffic reported)
timeout -k 10 420 python -u bench.py --config D > $O/bench_D.json 2> $O/bench_D.err
# config C's line again, now that pmc_latest.json is of this build (traffic reported)
timeout -k 10 300 python -u bench.py > $O/bench_C.json 2> $O/bench_C.err
# config E's line again, now that pmc_e.json is of this build (traffic reported)
timeout -k 10 900 python -u bench.py --config E > $O/bench_E.json 2> $O/bench_E.err
