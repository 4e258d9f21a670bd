#!/bin/bash
# Round 4: dedupe v3 (claim + classify passes, COUNT over the representatives
# only) — parity tests, then interleaved A/Bs on E (0.2), C and D.
set -o pipefail
mkdir -p gpurun_out/r04l
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "dedupe or group or config_e or deferred or global_stack or churn" > gpurun_out/r04l/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_match.py --config E --rounds 4 --opt dedupe=0,1 > gpurun_out/r04l/ab_E02.json 2> gpurun_out/r04l/ab_E02.err &&
timeout -k 10 240 python -u tools/ab_match.py --config C --rounds 4 --steps 16 --opt dedupe=0,2 > gpurun_out/r04l/ab_C.json 2> gpurun_out/r04l/ab_C.err &&
timeout -k 10 400 python -u tools/ab_match.py --config D --rounds 3 --steps 16 --opt dedupe=0,2 > gpurun_out/r04l/ab_D.json 2> gpurun_out/r04l/ab_D.err
