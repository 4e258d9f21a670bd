#!/bin/bash
# Round 5, session l: trie-less COUNT (R1, R2), auto lanes per publish (A),
# count_bpc 5; parity first, then the secondary lines.
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_word_lists.py -m gpu -k "trieless or r1 or exact_filter or heavy or verdict or churn_with_wild" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_C.json 2>/dev/null || exit 4
timeout -k 10 300 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e > $O/bench_R1.json 2>/dev/null || exit 5
timeout -k 10 300 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e --vmqg-opt trieless=0 > $O/bench_R1_tl0.json 2>/dev/null || exit 6
timeout -k 10 300 python bench.py --config R2 --r-n 4096000 --no-cpu-baseline --no-e2e > $O/bench_R2.json 2>/dev/null || exit 7
timeout -k 10 200 python bench.py --config A --no-cpu-baseline --no-e2e > $O/bench_A.json 2>/dev/null || exit 8
for f in $O/bench_*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read()); print('$(basename $f)', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"; done
