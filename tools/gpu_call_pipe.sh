#!/bin/bash
# pipelined match: GPU parity (new + existing match tests), then bench C
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_pipeline.py tests/test_gpu_parity.py > gpurun_out/pipe_tests.log 2>&1 || { tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -3 gpurun_out/pipe_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench_pipe.json 2> gpurun_out/bench_pipe.err || { tail -20 gpurun_out/bench_pipe.err; exit 1; }
cat gpurun_out/bench_pipe.json
