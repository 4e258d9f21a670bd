#!/bin/bash
# Round 4: atomic-cost probe; the defaults (dedupe and groups off) on C and D;
# the host harness with range-mode prefetch.
set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 60 tools/bin/atomic_probe > gpurun_out/r04h/atomic_probe.jsonl 2> gpurun_out/r04h/atomic_probe.err &&
timeout -k 10 240 python -u bench.py > gpurun_out/r04h/bench_C.json 2> gpurun_out/r04h/bench_C.err &&
timeout -k 10 420 python -u bench.py --config D > gpurun_out/r04h/bench_D.json 2> gpurun_out/r04h/bench_D.err &&
timeout -k 10 200 tools/bin/nif_harness 3 scale > gpurun_out/r04h/nif_harness.jsonl 2> gpurun_out/r04h/nif_harness.err
