#!/bin/bash
# Round-3: the GPU tests from test_wide_publishes_by_record_count on (the
# full suite stopped there), then the exact-filter A/B and the NIF harness.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03s}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_parity.py::test_wide_publishes_by_record_count" tests/test_host_engine.py tests/test_nif_layer.py tests/test_oracle_golden.py tests/test_retain.py tests/test_shared.py tests/test_workloads.py -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in default nofilter; do
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/c_$v.json 2> $O/c_$v.err || { tail -5 $O/c_$v.err; exit 3; }
  python3 -c "import json; d=json.load(open('$O/c_$v.json')); print('C $v', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})"
done
done
for v in default nofilter; do
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 300 python tools/ab_match.py --config D --rounds 2 --steps 10 > $O/d_$v.json 2> $O/d_$v.err || { tail -5 $O/d_$v.err; exit 4; }
  echo "D $v $(cat $O/d_$v.json)"
  VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 300 python tools/ab_match.py --config E --rounds 2 --steps 10 > $O/e_$v.json 2> $O/e_$v.err || { tail -5 $O/e_$v.err; exit 5; }
  echo "E $v $(cat $O/e_$v.json)"
done
timeout -k 10 400 tools/bin/nif_harness 2 > $O/nif.jsonl 2> $O/nif.err || { tail -5 $O/nif.err; exit 6; }
cat $O/nif.jsonl
echo done
