#!/bin/bash
# Round-3: which publishes go to the EMIT tail (VMQG_WIDE_RECORDS: >= 256
# records, or only > 8 keys) x fast_g, on config E at 0.2 scale and config D.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03n}
mkdir -p $O
for v in default norecwide; do
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 400 python tools/ab_match.py --config E --rounds 2 --steps 10 --opt fast_g=1,2 > $O/e_$v.json 2> $O/e_$v.err || { tail -5 $O/e_$v.err; exit 3; }
  echo "E $v $(cat $O/e_$v.json)"
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 300 python tools/ab_match.py --config D --rounds 2 --steps 10 > $O/d_$v.json 2> $O/d_$v.err || { tail -5 $O/d_$v.err; exit 4; }
  echo "D $v $(cat $O/d_$v.json)"
done
echo done
