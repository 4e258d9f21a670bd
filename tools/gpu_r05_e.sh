#!/bin/bash
# Round 5, session e: where heavy routing differs (diagnosis), then C's
# COUNT across builds interleaved, and R1 at 4,096,000.
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 240 python -u tools/diag_heavy.py > $O/diag.txt 2>&1 || { tail -30 $O/diag.txt; exit 3; }
cat $O/diag.txt
for rep in 1 2; do
for so in build/ab_r05/lib_*.so; do
  VMQG_LIB_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" >> $O/c_ab.txt || { echo "$so FAILED"; exit 4; }
done
done
cat $O/c_ab.txt
timeout -k 10 300 python -u bench.py --config R1 --r-n 4096000 --no-cpu-baseline > $O/bench_R1.json 2> $O/bench_R1.err
