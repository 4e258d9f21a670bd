#!/bin/bash
# final tree: the whole GPU suite, then config E at full size (50M subs)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests -m gpu > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 900 python -u bench.py --config E > gpurun_out/bench_E_final.json 2> gpurun_out/bench_E_final.err || { tail -20 gpurun_out/bench_E_final.err; exit 2; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_E_final.json')); print(d['value'], d.get('kernel_us'), (d.get('roofline') or {}).get('frac'))"
