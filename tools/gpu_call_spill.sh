# Key-spill A/B: parity tests on the new build, then configs C and E (0.2
# scale) with the spill (default) and without it (build/ab/lib_nospill.so),
# then the random-probe ceiling microbenchmark.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/spill_tests.log 2>&1 || { tail -30 $O/spill_tests.log; exit 3; }
tail -3 $O/spill_tests.log
for v in default nospill; do
  unset VMQG_LIB_PATH; [ $v = nospill ] && export VMQG_LIB_PATH=build/ab/lib_nospill.so
  timeout -k 10 300 python3 -u bench.py --config E --e-scale 0.2 --steps 10 --warmup 2 --no-cpu-baseline > $O/spill_E_$v.json 2> $O/spill_E_$v.err || { tail -20 $O/spill_E_$v.err; exit 4; }
  python3 -c "import json;d=json.load(open('$O/spill_E_$v.json'));print('$v E', d['value'], d['kernel_us'])"
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/spill_C_$v.json 2> $O/spill_C_$v.err || { tail -20 $O/spill_C_$v.err; exit 5; }
  python3 -c "import json;d=json.load(open('$O/spill_C_$v.json'));print('$v C', d['value'], d.get('kernel_us'))"
done
timeout -k 10 300 tools/bin/probe_ceiling > $O/probe_ceiling.jsonl 2>&1 || { tail -5 $O/probe_ceiling.jsonl; exit 6; }
cat $O/probe_ceiling.jsonl
