#!/bin/bash
# Round 5, session n: lazy second exact slot (general and exact-only COUNT),
# the tail's heavy loop with one-ahead loads (D, heavy_min 256, vs the build
# before it), then the secondary lines.
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_word_lists.py -m gpu -k "trieless or r1 or exact or heavy or config_d or verdict or wild" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
show() { python3 -c "import json,sys; d=json.loads(open('$1').read()); print('$(basename $1)', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"; }
timeout -k 10 300 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e > $O/bench_R1.json 2>/dev/null && show $O/bench_R1.json || exit 4
timeout -k 10 300 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e --vmqg-opt trieless=0 > $O/bench_R1_tl0.json 2>/dev/null && show $O/bench_R1_tl0.json || exit 5
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_C.json 2>/dev/null && show $O/bench_C.json || exit 6
for so in build/ab_r05/lib_cur.so build/ab_r05/lib_git_5309e6b.so; do
  VMQG_LIB_PATH=$so timeout -k 10 500 python bench.py --config D --no-cpu-baseline --no-e2e --vmqg-opt heavy_min=256 > $O/bench_D_h256_$(basename $so .so).json 2> $O/bench_D.err && show $O/bench_D_h256_$(basename $so .so).json || { tail -5 $O/bench_D.err; exit 7; }
done
timeout -k 10 500 python bench.py --config D --no-cpu-baseline --no-e2e > $O/bench_D_h0.json 2> $O/bench_D.err && show $O/bench_D_h0.json || exit 8
timeout -k 10 200 python bench.py --config A --no-cpu-baseline --no-e2e > $O/bench_A.json 2>/dev/null && show $O/bench_A.json || exit 9
