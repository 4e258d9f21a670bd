#!/bin/bash
# Round 4: dedupe with the claim pass — parity tests, then interleaved
# A/Bs of dedupe 0 / 1 / 2 on E (0.2), C and D.
set -o pipefail
mkdir -p gpurun_out/r04k
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "dedupe or group or config_e or config_d_churn or deferred or global_stack" > gpurun_out/r04k/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_match.py --config E --rounds 4 --opt dedupe=0,1,2 > gpurun_out/r04k/ab_E02.json 2> gpurun_out/r04k/ab_E02.err &&
timeout -k 10 240 python -u tools/ab_match.py --config C --rounds 4 --opt dedupe=0,2 > gpurun_out/r04k/ab_C.json 2> gpurun_out/r04k/ab_C.err &&
timeout -k 10 400 python -u tools/ab_match.py --config D --rounds 3 --opt dedupe=0,2 > gpurun_out/r04k/ab_D.json 2> gpurun_out/r04k/ab_D.err &&
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e > gpurun_out/r04k/bench_C.json 2> gpurun_out/r04k/bench_C.err
