#!/bin/bash
# Round 4 final build, call 3: config E at full size (50M subscriptions,
# oracle sample) and its LITE rocprofv3 session.
set -o pipefail
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 900 python -u bench.py --config E > $O/bench_E.json 2> $O/bench_E.err &&
LITE=1 OUT=$O/prof_E BENCH_ARGS="--config E" TAG=r04_E bash tools/profile_session.sh > $O/prof_E.log 2>&1
