#!/bin/bash
# Round 4: tier-2 stack hand-off A/B (fenced default vs the round-3 unfenced
# hand-off), then the global-stack test on the default build.
set -o pipefail
mkdir -p gpurun_out/r04t
timeout -k 10 300 python -u tools/diag_tier2.py 2048 3072 4096 > gpurun_out/r04t/tier2_fenced.txt 2>&1 &&
VMQG_LIB_PATH=build/ab/lib_nofence.so timeout -k 10 300 python -u tools/diag_tier2.py 3072 4096 > gpurun_out/r04t/tier2_nofence.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 250 --timeout-method thread -k "global_stack or frontier or deferred_tiers" > gpurun_out/r04t/tests.log 2>&1
