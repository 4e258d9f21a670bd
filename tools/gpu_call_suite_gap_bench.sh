#!/bin/bash
# full GPU suite, then a kernel-traced bench C with the gap report, then the bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gap6
timeout -k 10 900 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > gpurun_out/xpre_tests.log 2>&1 || { tail -30 gpurun_out/xpre_tests.log; exit 1; }
tail -2 gpurun_out/xpre_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gap6 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/gap6/bench.json 2> gpurun_out/gap6/bench.err || { tail -20 gpurun_out/gap6/bench.err; exit 2; }
f=$(find gpurun_out/gap6 -name "*kernel_trace.csv" | head -1)
python3 tools/gap_report.py $f > gpurun_out/gap6/report.json && cat gpurun_out/gap6/report.json && rm -f $f
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_xpre.json 2> gpurun_out/bench_xpre.err || { tail -20 gpurun_out/bench_xpre.err; exit 3; }
cat gpurun_out/bench_xpre.json
