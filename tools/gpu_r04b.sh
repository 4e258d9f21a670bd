#!/bin/bash
# Round 4, session b: the NIF C core on the GPU (combining submitter, the
# churn-that-changes-answers parity test), the host-half harness, and the
# full-size D / 0.2-scale E parity tests.
set -o pipefail
mkdir -p gpurun_out/r04b
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_nif_layer.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b/nif_tests.log 2>&1 &&
timeout -k 10 400 tools/bin/nif_harness 3 > gpurun_out/r04b/nif_harness.jsonl 2> gpurun_out/r04b/nif_harness.err &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 500 --timeout-method thread -k "full_size_under_churn or scale_02" > gpurun_out/r04b/big_tests.log 2>&1
