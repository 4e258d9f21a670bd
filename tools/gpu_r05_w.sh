#!/bin/bash
# Round 5, session w (final build, no library change): the random-probe
# ceiling re-measured on today's pool, R1's and A's instruction / wait mix
# (SQ counters) and R1's L2 / memory-side requests, for the R1 request-rate
# roofline in DESIGN.md and next round's A work.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 180 ./tools/bin/probe_ceiling > $O/probe_ceiling.jsonl 2> $O/probe_ceiling.err || { tail -5 $O/probe_ceiling.err; exit 3; }
tail -3 $O/probe_ceiling.jsonl
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_R1 -o run --output-format csv -- python3 bench.py --config R1 --r-n 4096000 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/sq_R1.log 2>&1 || { tail -5 $O/sq_R1.log; exit 4; }
timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_A -o run --output-format csv -- python3 bench.py --config A --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/sq_A.log 2>&1 || { tail -5 $O/sq_A.log; exit 5; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/l2_R1 -o run --output-format csv -- python3 bench.py --config R1 --r-n 4096000 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/l2_R1.log 2>&1 || { tail -5 $O/l2_R1.log; exit 6; }
find $O -name "*counter_collection.csv" | head
