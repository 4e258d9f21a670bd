#!/bin/bash
# Round 4, session a: headline C with uninstrumented timing + median, the
# reference-shaped R1/R2 lines at N = 4,096,000 and a config A line.
set -o pipefail
mkdir -p gpurun_out/r04a
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py > gpurun_out/r04a/bench_C.json 2> gpurun_out/r04a/bench_C.log &&
timeout -k 10 300 python -u bench.py --config R1 --r-n 4096000 > gpurun_out/r04a/bench_R1.json 2> gpurun_out/r04a/bench_R1.log &&
timeout -k 10 300 python -u bench.py --config R2 --r-n 4096000 > gpurun_out/r04a/bench_R2.json 2> gpurun_out/r04a/bench_R2.log &&
timeout -k 10 300 python -u bench.py --config A > gpurun_out/r04a/bench_A.json 2> gpurun_out/r04a/bench_A.log &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04a/gpu_tests.log 2>&1
