#!/bin/bash
# Round 5, session i: C's COUNT with the exact-lookup counters as packed
# lane counters (default) vs off vs per-wave ballots; R1's and C's COUNT
# instruction / wait mix (SQ counters) and R1's L2 behaviour.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
for rep in 1 2; do
for so in build/ab_r05/lib_*.so; do
  VMQG_LIB_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" >> $O/c_ab.txt || { echo "$so FAILED"; exit 4; }
done
done
cat $O/c_ab.txt
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_R1 -o run --output-format csv -- python3 bench.py --config R1 --r-n 4096000 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/sq_R1.log 2>&1 || { tail -5 $O/sq_R1.log; exit 5; }
timeout -s KILL 240 rocprofv3 --pmc $SQ -d $O/sq_C -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/sq_C.log 2>&1 || { tail -5 $O/sq_C.log; exit 6; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/l2_R1 -o run --output-format csv -- python3 bench.py --config R1 --r-n 4096000 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-timing > $O/l2_R1.log 2>&1 || { tail -5 $O/l2_R1.log; exit 7; }
ls -R $O | head -40
