#!/bin/bash
# build v13 (one-lane COUNT): PMC session, then the whole GPU suite, a
# kernel-traced bench C with the gap report, the bench lines of C, D and E
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/v13
TAG=r02_v13 OUT=gpurun_out/v13/prof bash tools/profile_session.sh > gpurun_out/v13/prof.log 2>&1 || { tail -20 gpurun_out/v13/prof.log; exit 1; }
cp gpurun_out/v13/prof/pmc_summary.json profiles/pmc_latest.json
timeout -k 10 900 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > gpurun_out/v13/tests.log 2>&1 || { tail -30 gpurun_out/v13/tests.log; exit 2; }
tail -2 gpurun_out/v13/tests.log
mkdir -p gpurun_out/v13/gap
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/v13/gap -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/v13/gap/bench.json 2> gpurun_out/v13/gap/bench.err || { tail -20 gpurun_out/v13/gap/bench.err; exit 3; }
f=$(find gpurun_out/v13/gap -name "*kernel_trace.csv" | head -1)
python3 tools/gap_report.py $f > gpurun_out/v13/gap_report.json && cat gpurun_out/v13/gap_report.json && rm -rf gpurun_out/v13/gap
timeout -k 10 400 python3 bench.py > gpurun_out/v13/bench_C.json 2> gpurun_out/v13/bench_C.err || { tail -20 gpurun_out/v13/bench_C.err; exit 4; }
cat gpurun_out/v13/bench_C.json
timeout -k 10 400 python3 bench.py --config D > gpurun_out/v13/bench_D.json 2> gpurun_out/v13/bench_D.err || { tail -20 gpurun_out/v13/bench_D.err; exit 5; }
timeout -k 10 900 python3 bench.py --config E > gpurun_out/v13/bench_E.json 2> gpurun_out/v13/bench_E.err || { tail -20 gpurun_out/v13/bench_E.err; exit 6; }
for c in D E; do python3 -c "import json; d=json.load(open('gpurun_out/v13/bench_$c.json')); r=d.get('roofline') or {}; print('$c', '%.3g'%d['value'], d.get('kernel_us'), 'frac', r.get('frac'))"; done
