#!/bin/bash
# Round 5, session r: trie-less EMIT (k_emit_exact) and the EMIT tail's
# wide-publish split, on the candidate in-tree build: the GPU tests that
# reach them, then R1 / A / R2 bench A/Bs against the frozen build
# (build/abx/lib_frozen.so) and knob variants.
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "trieless or r1_r2 or wide or heavy or many_key or offsets or retry" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
[ -n "$SKIP_TESTS" ] || tail -2 $O/tests.log
b() {  # label, lib ('' = in-tree), bench args
  local lab=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then export VMQG_LIB_PATH=$lib; else unset VMQG_LIB_PATH; fi
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e "$@" > $O/b_$lab.json 2> $O/b_$lab.err || { tail -5 $O/b_$lab.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/b_$lab.json')); print('$lab', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()}, (d.get('oracle_sample') or {}).get('differ'))" | tee -a $O/ab.txt
}
unset VMQG_LIB_PATH
R1="--config R1 --r-n 4096000"
b R1_new "" $R1 && b R1_frozen build/abx/lib_frozen.so $R1 && b R1_k2 build/abx/lib_emitexk2.so $R1 && \
b R1_k8 build/abx/lib_emitexk8.so $R1 && b R1_new2 "" $R1 && b R1_frozen2 build/abx/lib_frozen.so $R1 || exit 4
b A_new "" --config A && b A_frozen build/abx/lib_frozen.so --config A && b A_nosplit build/abx/lib_nosplit.so --config A && \
b A_new2 "" --config A && b A_frozen2 build/abx/lib_frozen.so --config A && b A_nosplit2 build/abx/lib_nosplit.so --config A || exit 5
b R2_new "" --config R2 --r-n 4096000 && b R2_frozen build/abx/lib_frozen.so --config R2 --r-n 4096000 || exit 6
unset VMQG_LIB_PATH
timeout -k 10 200 python -u tools/ab_match.py --config A --opt dedupe=0,2 > $O/ab_A_dedupe.json 2> $O/ab_A_dd.err || { tail -5 $O/ab_A_dd.err; exit 7; }
cat $O/ab_A_dedupe.json
