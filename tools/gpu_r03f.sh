#!/bin/bash
# Round-3: the whole -m gpu suite, then config D's EMIT tail under the
# build/ab variants (two wide publishes per wave or one; XCD labels or chunk
# owners), then config C on the in-tree library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03j}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for v in default noxcd wide64 wide64_noxcd; do
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 300 python tools/ab_match.py --config D --rounds 2 --steps 10 > $O/d_$v.json 2> $O/d_$v.err || { tail -5 $O/d_$v.err; exit 3; }
  echo "D $v $(cat $O/d_$v.json)"
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e > $O/bench_C.json 2> $O/bench_C.err || { tail -5 $O/bench_C.err; exit 4; }
python3 -c "import json; d=json.load(open('$O/bench_C.json')); print('C', '%.4g' % d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"
echo done
