# '#'-alias A/B: parity tests on the new build, then config C and config E
# (0.2 scale) under the default build and the variants named in $VARIANTS
# (build/ab/lib_<name>.so, tools/build_variants.py), interleaved, twice.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/alias_tests.log 2>&1 || { tail -30 $O/alias_tests.log; exit 3; }
[ -n "$SKIP_TESTS" ] || tail -2 $O/alias_tests.log
for rep in 1 2; do
  for v in default ${VARIANTS:-noalias}; do
    unset VMQG_LIB_PATH; [ $v != default ] && export VMQG_LIB_PATH=build/ab/lib_$v.so
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/alias_C_${v}_$rep.json 2> $O/alias_C_${v}_$rep.err || { tail -20 $O/alias_C_${v}_$rep.err; exit 5; }
    python3 -c "import json;d=json.load(open('$O/alias_C_${v}_$rep.json'));print('$v C', d['value'], d.get('kernel_us'))"
  done
done
for v in default ${VARIANTS:-noalias}; do
  unset VMQG_LIB_PATH; [ $v != default ] && export VMQG_LIB_PATH=build/ab/lib_$v.so
  timeout -k 10 300 python3 -u bench.py --config E --e-scale 0.2 --steps 10 --warmup 2 --no-cpu-baseline > $O/alias_E_$v.json 2> $O/alias_E_$v.err || { tail -20 $O/alias_E_$v.err; exit 4; }
  python3 -c "import json;d=json.load(open('$O/alias_E_$v.json'));print('$v E', d['value'], d['kernel_us'], d['arena_bytes'])"
done
[ -n "$SKIP_PROBE" ] || timeout -k 10 300 tools/bin/probe_ceiling > $O/probe_ceiling.jsonl 2>&1 || { tail -5 $O/probe_ceiling.jsonl; exit 6; }
[ -n "$SKIP_PROBE" ] || cat $O/probe_ceiling.jsonl
