#!/bin/bash
# Round 4 final build, call 1: the whole GPU suite, smoke(), the headline line.
set -o pipefail
O=gpurun_out/final1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_C.json 2> $O/bench_C.err
