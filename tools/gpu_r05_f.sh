#!/bin/bash
# Round 5, session f: the whole GPU suite after the reader/writer split
# (apply stage/commit, readers' record buffers, lock-free dictionary), the
# NIF harness (scale, windowed churn, load), and C's COUNT across builds.
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -3 $O/tests.log
timeout -k 10 420 ./tools/bin/nif_harness 3 scale churn load > $O/harness.jsonl 2> $O/harness.err || { tail -20 $O/harness.err; exit 4; }
for rep in 1 2; do
for so in build/ab_r05/lib_*.so; do
  VMQG_LIB_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" >> $O/c_ab.txt || { echo "$so FAILED"; exit 5; }
done
done
cat $O/c_ab.txt
