#!/bin/bash
# Round 4: block-aggregated COUNT counters / deferred list and tail totals —
# parity tests on the paths they touch, then C, D and E (0.2, A/B tool) timings.
set -o pipefail
mkdir -p gpurun_out/r04i
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "deferred or frontier or wide or dedupe or group or config_d or config_e or global_stack or churn" > gpurun_out/r04i/tests.log 2>&1 &&
timeout -k 10 240 python -u bench.py > gpurun_out/r04i/bench_C.json 2> gpurun_out/r04i/bench_C.err &&
timeout -k 10 420 python -u bench.py --config D > gpurun_out/r04i/bench_D.json 2> gpurun_out/r04i/bench_D.err &&
timeout -k 10 300 python -u tools/ab_match.py --config E --rounds 3 --opt dedupe=0 > gpurun_out/r04i/ab_E02.json 2> gpurun_out/r04i/ab_E02.err
