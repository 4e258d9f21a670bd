#!/bin/bash
# Round 5, session k: the exact-filter sampler build (COUNT tracks nothing):
# the filter tests, C and R1 with 4 / 5 COUNT blocks per CU, R1 at 1M; then
# heavy-publish routing on D and E and A's lanes per publish (session j).
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "exact_filter or heavy or r1 or R1" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for bpc in 4 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --vmqg-opt count_bpc=$bpc > $O/bench_C_bpc$bpc.json 2>/dev/null || exit 4
  timeout -k 10 300 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e --vmqg-opt count_bpc=$bpc > $O/bench_R1_bpc$bpc.json 2>/dev/null || exit 5
done
timeout -k 10 300 python bench.py --config R1 --r-n 1000000 --no-cpu-baseline --no-e2e > $O/bench_R1_1M.json 2>/dev/null || exit 6
for f in $O/bench_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read()); print('$(basename $f)', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"; done
bash tools/gpu_r05_j.sh
