#!/bin/bash
# Round 4 final build, call 1: the whole GPU suite, then config E's line at
# full size (50M subscriptions, oracle sample, CPU baseline).
set -o pipefail
O=gpurun_out/final1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 900 python -u bench.py --config E > $O/bench_E.json 2> $O/bench_E.err
