#!/bin/bash
# Round 5, session s: k_emit_exact blocks per wave (1 / 2 / 4) on R1, the
# dedupe auto threshold (50 % vs 67 %) on A and D, after the trie-less and
# wide-publish GPU tests on the candidate in-tree build.
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "trieless or r1_r2 or wide or heavy or many_key or offsets or retry or dedupe" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
b() {  # label, lib ('' = in-tree), bench args
  local lab=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export VMQG_LIB_PATH=$lib; else unset VMQG_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e "$@" > $O/b_$lab.json 2> $O/b_$lab.err || { tail -5 $O/b_$lab.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/b_$lab.json')); print('$lab', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()}, d.get('served'))" | tee -a $O/ab.txt
}
R1="--config R1 --r-n 4096000"
b R1_k2 "" $R1 && b R1_k1 build/abx/lib_emitexk1.so $R1 && b R1_k4 build/abx/lib_emitexk4.so $R1 && b R1_k2b "" $R1 || exit 4
b A_50 "" --config A && b A_67 build/abx/lib_ddpct67.so --config A && b A_50b "" --config A && b A_67b build/abx/lib_ddpct67.so --config A || exit 5
b D_50 "" --config D && b D_67 build/abx/lib_ddpct67.so --config D || exit 6
