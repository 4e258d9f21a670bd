#!/bin/bash
# Round 4: dedupe v3 with the parallel fix-up pass and 4-lane representatives:
# dedupe tests, then interleaved A/Bs on E (0.2), C and D (auto mode).
set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "dedupe or config_e or deferred or global_stack" > gpurun_out/r04m/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/ab_match.py --config E --rounds 3 --opt dedupe=0,1 > gpurun_out/r04m/ab_E02.json 2> gpurun_out/r04m/ab_E02.err &&
timeout -k 10 240 python -u tools/ab_match.py --config C --rounds 3 --steps 64 --opt dedupe=0,2 > gpurun_out/r04m/ab_C.json 2> gpurun_out/r04m/ab_C.err &&
timeout -k 10 400 python -u tools/ab_match.py --config D --rounds 2 --steps 32 --opt dedupe=0,2 > gpurun_out/r04m/ab_D.json 2> gpurun_out/r04m/ab_D.err
