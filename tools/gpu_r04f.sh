#!/bin/bash
# Round 4, session f: config E at full size (50M subscriptions, batch dedupe).
set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 900 python -u bench.py --config E > gpurun_out/r04f/bench_E.json 2> gpurun_out/r04f/bench_E.err
