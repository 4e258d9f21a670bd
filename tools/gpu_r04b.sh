#!/bin/bash
# Round 4, session b: the NIF C core on the GPU (combining submitter, the
# churn-that-changes-answers check, the NIF glue over the erl_nif double),
# the host-half harness, then the whole GPU suite (incl. full-size D,
# 0.2-scale E, batch dedupe).
set -o pipefail
mkdir -p gpurun_out/r04b
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_nif_layer.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b/nif_tests.log 2>&1 &&
timeout -k 10 300 tools/bin/nif_harness 3 > gpurun_out/r04b/nif_harness.jsonl 2> gpurun_out/r04b/nif_harness.err &&
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --deselect tests/test_nif_layer.py > gpurun_out/r04b/gpu_tests.log 2>&1
