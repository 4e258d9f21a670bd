#!/bin/bash
# Round 4, session d: the whole GPU suite, the host-half harness (scale with
# span folds, three rounds in flight), the default bench line.
set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r04d/gpu_tests.log 2>&1 &&
timeout -k 10 200 tools/bin/nif_harness 3 scale inflight > gpurun_out/r04d/nif_harness.jsonl 2> gpurun_out/r04d/nif_harness.err &&
timeout -k 10 200 python -u bench.py > gpurun_out/r04d/bench_C.json 2> gpurun_out/r04d/bench_C.err
