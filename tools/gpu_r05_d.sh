#!/bin/bash
# Round 5, session d: C's COUNT on the round-4 build vs this round's builds,
# interleaved on one box; D with the XCD-routed heavy publishes at several
# thresholds; R1 with its exact table at load 0.5; the heavy / filter parity
# tests.
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "heavy or exact_filter" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
for rep in 1 2; do
for so in build/ab_r05/lib_*.so; do
  VMQG_LIB_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" >> $O/c_ab.txt || { echo "$so FAILED"; exit 4; }
done
done
cat $O/c_ab.txt
for hm in 0 256 128 1024; do
  timeout -k 10 420 python -u bench.py --config D --no-cpu-baseline --vmqg-opt heavy_min=$hm > $O/bench_D_h$hm.json 2> $O/bench_D_h$hm.err || exit 5
done
timeout -k 10 300 python -u bench.py --config R1 --r-n 4096000 --no-cpu-baseline > $O/bench_R1.json 2> $O/bench_R1.err
