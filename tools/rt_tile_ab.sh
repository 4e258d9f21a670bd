#!/bin/bash
# Retained-walk tile/unroll A/B (build/ab from tools/build_variants.py), the
# retained parity tests on each variant, then rocprofv3 sessions (kernel
# trace + PMC) of RT, AC and SS on the default build (build-tagged summaries).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r04rt}
mkdir -p $O
for v in default rt_tile256 rt_tile512 rt_tile2048 rt_u8 default; do
  so=build/ab/lib_$v.so
  for rep in 1; do
    J=$O/rt_$v.$SECONDS.json
    VMQG_LIB_PATH=$so timeout -k 10 120 python3 bench.py --config RT --steps 30 --warmup 3 --no-cpu-baseline > $J 2> $O/rt_$v.err || { tail -5 $O/rt_$v.err; exit 2; }
    python3 -c "import json; d=json.load(open('$J')); print('$v', '%.4g'%d['value'], round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"
  done
done
for v in rt_tile256 rt_tile512 rt_tile2048; do
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_retain.py -m gpu > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 3; }
  echo "$v tests: $(tail -1 $O/tests_$v.log)"
done
[ -n "${NOPROF:-}" ] && { echo done; exit 0; }   # NOPROF=1: the A/B and tests only
for c in RT AC SS; do
  LITE=1 OUT=$O/prof_$c BENCH_ARGS="--config $c" TAG=r04_$c bash tools/profile_session.sh > $O/prof_$c.log 2>&1 || { tail -20 $O/prof_$c.log; exit 4; }
  tail -3 $O/prof_$c.log
done
echo done
