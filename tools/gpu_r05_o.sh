#!/bin/bash
# Round 5, session o: where D's EMIT tail (heavy routing) and E's fast EMIT
# spend their time: HBM bytes per kernel and the SQ instruction / wait mix.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
OUT=$O/prof_D LITE=1 TAG=r05_D_h256 BENCH_ARGS="--config D --vmqg-opt heavy_min=256" timeout -k 10 900 bash tools/profile_session.sh > $O/prof_D.log 2>&1 || { tail -5 $O/prof_D.log; exit 3; }
tail -2 $O/prof_D.log
timeout -s KILL 400 rocprofv3 --pmc $SQ -d $O/sq_D -o run --output-format csv -- python3 bench.py --config D --vmqg-opt heavy_min=256 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/sq_D.log 2>&1 || { tail -5 $O/sq_D.log; exit 4; }
timeout -s KILL 500 rocprofv3 --pmc $SQ -d $O/sq_E -o run --output-format csv -- python3 bench.py --config E --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/sq_E.log 2>&1 || { tail -5 $O/sq_E.log; exit 5; }
timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_C -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/sq_C.log 2>&1 || { tail -5 $O/sq_C.log; exit 6; }
