#!/bin/bash
# Round 5, session u: exact slots per topic 2 vs 4 (library knob
# VMQG_EXACT_SLOTS_PER_TOPIC) on E, D and R1 before it becomes the default.
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
b() {  # label, lib, bench args
  local lab=$1 lib=$2; shift 2
  VMQG_LIB_PATH=$lib timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e "$@" > $O/b_$lab.json 2> $O/b_$lab.err || { tail -5 $O/b_$lab.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/b_$lab.json')); print('$lab', '%.4g' % d['value'], d.get('arena_bytes'), {k: round(v,1) for k,v in d['kernel_us'].items()}, (d.get('oracle_sample') or {}).get('differ'), d.get('load_s'))" | tee -a $O/ab.txt
}
b R1_2 build/abu/lib_default.so --config R1 --r-n 4096000 && b R1_4 build/abu/lib_exact4x.so --config R1 --r-n 4096000 || exit 3
b D_2 build/abu/lib_default.so --config D && b D_4 build/abu/lib_exact4x.so --config D || exit 4
b E_2 build/abu/lib_default.so --config E && b E_4 build/abu/lib_exact4x.so --config E || exit 5
