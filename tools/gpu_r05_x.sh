#!/bin/bash
# Round 5, session x: a 16-B key cache for trie-less COUNT -> EMIT (an
# out-of-tree variant, build/abw/lib_kc16.so): its trie-less parity tests,
# then R1 against the in-tree build.
set -o pipefail
O=gpurun_out/r05x
mkdir -p $O
VMQG_LIB_PATH=build/abw/lib_kc16.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_word_lists.py -m gpu -k "trieless or r1_r2 or word or wild" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
b() {  # label, lib ('' = in-tree), bench args
  local lab=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export VMQG_LIB_PATH=$lib; else unset VMQG_LIB_PATH; fi
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e "$@" > $O/b_$lab.json 2> $O/b_$lab.err || { tail -5 $O/b_$lab.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/b_$lab.json')); print('$lab', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" | tee -a $O/ab.txt
}
R1="--config R1 --r-n 4096000"
b R1_base "" $R1 && b R1_kc16 build/abw/lib_kc16.so $R1 && b R1_base2 "" $R1 && b R1_kc16b build/abw/lib_kc16.so $R1 || exit 4
b R2_kc16 build/abw/lib_kc16.so --config R2 --r-n 4096000 || exit 5
