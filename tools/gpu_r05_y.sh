#!/bin/bash
# Round 5, session y: the NIF harness and the N = 2 launcher-less rehearsal
# again on the final build 4b4af682.
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 420 ./tools/bin/nif_harness 3 scale churn load > $O/harness.jsonl 2> $O/harness.err || { tail -20 $O/harness.err; exit 3; }
tail -3 $O/harness.jsonl
timeout -k 10 300 python -u bench.py --gpus 2 --force-device 0 --dist-backend gloo --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_C_n2.json 2> $O/bench_C_n2.err || { tail -5 $O/bench_C_n2.err; exit 4; }
tail -c 300 $O/bench_C_n2.json
