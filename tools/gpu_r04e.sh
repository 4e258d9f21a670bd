#!/bin/bash
# Round 4, session e: host-half harness, the headline line, R2 at the
# reference suite's N = 4,096,000 (huge-publish segments), D at full size
# (output groups).  E runs in its own call (tools/gpu_r04f.sh).
set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 300 tools/bin/nif_harness 3 scale inflight churn load > gpurun_out/r04e/nif_harness.jsonl 2> gpurun_out/r04e/nif_harness.err &&
timeout -k 10 240 python -u bench.py > gpurun_out/r04e/bench_C.json 2> gpurun_out/r04e/bench_C.err &&
timeout -k 10 240 python -u bench.py --config R2 --r-n 4096000 > gpurun_out/r04e/bench_R2.json 2> gpurun_out/r04e/bench_R2.err &&
timeout -k 10 420 python -u bench.py --config D > gpurun_out/r04e/bench_D.json 2> gpurun_out/r04e/bench_D.err
