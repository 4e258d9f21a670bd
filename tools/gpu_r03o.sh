#!/bin/bash
# Short retained-walk tile A/B: RT bench on the default build and the 256-,
# 512- and 2,048-row tile variants (build/ab from tools/build_variants.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03o}
mkdir -p $O
for v in default rt_tile256 rt_tile512 rt_tile2048 default; do
  J=$O/rt_$v.$SECONDS.json
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 120 python3 bench.py --config RT --steps 30 --warmup 3 --no-cpu-baseline > $J 2> $O/rt_$v.err || { tail -5 $O/rt_$v.err; exit 2; }
  python3 -c "import json; d=json.load(open('$J')); print('$v', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"
done
echo done
