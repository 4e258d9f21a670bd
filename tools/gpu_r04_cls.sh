#!/bin/bash
# Classify with wave ballots and batched word loads: dedupe tests, then E.
set -o pipefail
O=gpurun_out/cls
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "dedupe or config_e or dollar or deferr" > $O/gpu_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --config E --no-cpu-baseline > $O/bench_E.json 2> $O/bench_E.err
