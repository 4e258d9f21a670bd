#!/bin/bash
# Round 4, session e: the secondary bench lines on the shipped build —
# R2 at the reference suite's N = 4,096,000 (huge-publish segments), D at
# full size (output groups), E at full size (batch dedupe).
set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 240 python -u bench.py --config R2 --r-n 4096000 > gpurun_out/r04e/bench_R2.json 2> gpurun_out/r04e/bench_R2.err &&
timeout -k 10 420 python -u bench.py --config D > gpurun_out/r04e/bench_D.json 2> gpurun_out/r04e/bench_D.err &&
timeout -k 10 500 python -u bench.py --config E > gpurun_out/r04e/bench_E.json 2> gpurun_out/r04e/bench_E.err
