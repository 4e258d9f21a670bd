#!/bin/bash
# Round-3: EMIT tail grid (blocks per CU) A/B — config C (the empty tail's
# launch cost) and config D (the tail's wide publishes) per build/ab variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03k}
mkdir -p $O
for v in ${VARIANTS:-default tail3 tail4 tail8}; do
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/c_$v.json 2> $O/c_$v.err || { tail -5 $O/c_$v.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/c_$v.json')); print('C $v', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 300 python tools/ab_match.py --config D --rounds 2 --steps 10 > $O/d_$v.json 2> $O/d_$v.err || { tail -5 $O/d_$v.err; exit 4; }
  echo "D $v $(cat $O/d_$v.json)"
done
echo done
