#!/bin/bash
# Round 4 final build, call 3: config E's LITE rocprofv3 session (kernel
# trace + FETCH/WRITE; each pass loads the 50M subscriptions again).
set -o pipefail
O=gpurun_out/final3
mkdir -p $O
LITE=1 OUT=$O/prof_E BENCH_ARGS="--config E" TAG=r04_E bash tools/profile_session.sh > $O/prof_E.log 2>&1
