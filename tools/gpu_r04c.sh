#!/bin/bash
# Round 4, session c: the E 0.2 output check in the parity test's order, then
# the big-config and dedupe / output-group parity tests in one process.
set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 300 python -u tools/diag_holes.py 0.2 > gpurun_out/r04c/holes2.jsonl 2> gpurun_out/r04c/holes2.err &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "config_d_full or config_e_scale or group_slots or dedupe or output_groups" > gpurun_out/r04c/tests.log 2>&1
