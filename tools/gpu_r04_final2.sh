#!/bin/bash
# Round 4 final build, call 2: smoke(), the headline line, its rocprofv3
# session (kernel trace + FETCH/WRITE + L2 + LDS passes), then config D's
# line and its LITE session (kernel trace + FETCH/WRITE).
set -o pipefail
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_C.json 2> $O/bench_C.err &&
OUT=$O/prof_C TAG=r04_C bash tools/profile_session.sh > $O/prof_C.log 2>&1 &&
timeout -k 10 420 python -u bench.py --config D > $O/bench_D.json 2> $O/bench_D.err &&
LITE=1 OUT=$O/prof_D BENCH_ARGS="--config D" TAG=r04_D bash tools/profile_session.sh > $O/prof_D.log 2>&1
