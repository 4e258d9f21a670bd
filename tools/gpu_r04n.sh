#!/bin/bash
# Round 4: dedupe auto by default — the whole GPU suite, then C and E lines.
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --no-e2e --no-cpu-baseline > $O/bench_C.json 2> $O/bench_C.err &&
timeout -k 10 600 python -u bench.py --config E --no-cpu-baseline > $O/bench_E.json 2> $O/bench_E.err
