#!/bin/bash
# Round 5, session g: after the fix of session f's fault (match calls read
# the device layout, not the layout a concurrent stage is re-laying out):
# the writer test with a table-growing group first, then the harness's load
# and churn sections, then the whole GPU suite, then A/B runs.
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_nif_layer.py -m gpu > $O/nif_tests.log 2>&1 || { tail -30 $O/nif_tests.log; exit 3; }
tail -2 $O/nif_tests.log
timeout -k 10 300 ./tools/bin/nif_harness 3 load churn > $O/harness_lc.jsonl 2> $O/harness_lc.err || { tail -20 $O/harness_lc.err; exit 4; }
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 5; }
tail -2 $O/tests.log
for rep in 1 2; do
for so in build/ab_r05/lib_*.so; do
  VMQG_LIB_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" >> $O/c_ab.txt || { echo "$so FAILED"; exit 6; }
done
done
cat $O/c_ab.txt
for rf in 1 0; do
  timeout -k 10 300 python -u bench.py --config R1 --r-n 4096000 --no-cpu-baseline --vmqg-opt root_flags=$rf > $O/bench_R1_rf$rf.json 2> $O/bench_R1_rf$rf.err || exit 7
done
