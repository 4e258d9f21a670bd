#!/bin/bash
# Round 4 final build, call 7: config E's full rocprofv3 session (adds the
# L2 hit/miss and LDS passes to call 3's LITE one).
set -o pipefail
O=gpurun_out/final7
mkdir -p $O
OUT=$O/prof_E BENCH_ARGS="--config E" TAG=r04_E bash tools/profile_session.sh > $O/prof_E.log 2>&1
