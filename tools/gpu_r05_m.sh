#!/bin/bash
# Round 5, session m: the GPU parity suite on the 3..4-key EMIT path and the
# exact-only COUNT reading slots in 16-B quarters; R1 trieless on / off with
# L2 requests; E with the new EMIT vs without (A/B libraries).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_word_lists.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for tl in 1 0; do
  timeout -k 10 300 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e --vmqg-opt trieless=$tl > $O/bench_R1_tl$tl.json 2>/dev/null || exit 4
  python3 -c "import json,sys; d=json.loads(open('$O/bench_R1_tl$tl.json').read()); print('R1 tl$tl', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $O/l2_R1_tl$tl -o run --output-format csv -- python3 bench.py --config R1 --r-n 4096000 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-timing --vmqg-opt trieless=$tl > $O/l2_R1_tl$tl.log 2>&1 || { tail -5 $O/l2_R1_tl$tl.log; exit 5; }
done
for so in build/ab_r05/lib_default.so build/ab_r05/lib_emitk4_0.so; do
  VMQG_LIB_PATH=$so timeout -k 10 500 python bench.py --config E --no-cpu-baseline --no-e2e > $O/bench_E_$(basename $so .so).json 2> $O/bench_E.err || { tail -5 $O/bench_E.err; exit 6; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_E_$(basename $so .so).json').read()); print('E $(basename $so)', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"
done
