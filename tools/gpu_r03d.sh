#!/bin/bash
# Round-3 A/B session over build/ab variants (tools/build_variants.py):
# config C step and kernel times, config D (tools/ab_match.py) per variant,
# the shared-subscription dispatch (SS) with and without the kind pre-pass,
# and the shared-subscription GPU tests on the in-tree library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03h}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_shared.py -m gpu > $O/ss_tests.log 2>&1 || { tail -30 $O/ss_tests.log; exit 2; }
tail -1 $O/ss_tests.log
for v in default tail8 walkinline; do
  so=build/ab/lib_$v.so
  VMQG_LIB_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/c_$v.json 2> $O/c_$v.err || { tail -5 $O/c_$v.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/c_$v.json')); print('C $v', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"
  VMQG_LIB_PATH=$so timeout -k 10 300 python tools/ab_match.py --config D --rounds 2 --steps 10 > $O/d_$v.json 2> $O/d_$v.err || { tail -5 $O/d_$v.err; exit 4; }
  echo "D $v $(cat $O/d_$v.json)"
done
for v in default ss_nokind; do
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 400 python bench.py --config SS --no-cpu-baseline > $O/ss_$v.json 2> $O/ss_$v.err || { tail -5 $O/ss_$v.err; exit 5; }
  python3 -c "import json; d=json.load(open('$O/ss_$v.json')); print('SS $v', '%.4g' % d['value'], d.get('kernel_us'), d['roofline'].get('frac'))"
done
echo done
