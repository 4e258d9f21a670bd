#!/bin/bash
# Round 5, session h: C's COUNT with the exact-lookup counters / the runtime
# filter switch compiled out (interleaved), A with 1 / 2 / 4 lanes per
# publish, E's output shape at 0.2 scale, R1's COUNT traffic (FETCH/WRITE).
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
for rep in 1 2; do
for so in build/ab_r05/lib_*.so; do
  VMQG_LIB_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" >> $O/c_ab.txt || { echo "$so FAILED"; exit 4; }
done
done
cat $O/c_ab.txt
for g in 1 2 4; do
  timeout -k 10 200 python -u bench.py --config A --no-cpu-baseline --no-e2e --fast-g $g > $O/bench_A_g$g.json 2> $O/bench_A_g$g.err || exit 5
done
timeout -k 10 300 python -u tools/diag_shape.py E 0.2 > $O/diag_E.txt 2>&1 || { tail -5 $O/diag_E.txt; exit 6; }
cat $O/diag_E.txt
OUT=$O/prof_R1 LITE=1 TAG=r05_R1 BENCH_ARGS="--config R1 --r-n 4096000" timeout -k 10 600 bash tools/profile_session.sh > $O/prof_R1.log 2>&1 || { tail -5 $O/prof_R1.log; exit 7; }
tail -3 $O/prof_R1.log
