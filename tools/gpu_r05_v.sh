#!/bin/bash
# Round 5, session v: four exact slots per topic with the filter kept at one
# bit per two slots' worth (D's filter stays L2-sized) vs the default, on D and R1.
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
b() {  # label, lib, bench args
  local lab=$1 lib=$2; shift 2
  VMQG_LIB_PATH=$lib timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e "$@" > $O/b_$lab.json 2> $O/b_$lab.err || { tail -5 $O/b_$lab.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/b_$lab.json')); print('$lab', '%.4g' % d['value'], d.get('arena_bytes'), {k: round(v,1) for k,v in d['kernel_us'].items()})" | tee -a $O/ab.txt
}
b D_2 build/abu/lib_default.so --config D && b D_4b2 build/abu/lib_exact4x_b2.so --config D && \
b D_2b build/abu/lib_default.so --config D && b D_4b2b build/abu/lib_exact4x_b2.so --config D || exit 3
b R1_4b2 build/abu/lib_exact4x_b2.so --config R1 --r-n 4096000 && b A_4b2 build/abu/lib_exact4x_b2.so --config A && b A_2 build/abu/lib_default.so --config A || exit 4
