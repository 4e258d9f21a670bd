#!/bin/bash
# Round 6, final session 5: the N = 2 launcher-less rehearsal (both ranks on
# this box's one GPU, gloo for both groups), C and D.
set -o pipefail
O=gpurun_out/r06f5
mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 2 --force-device 0 --dist-backend gloo --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_C_n2.json 2> $O/bench_C_n2.err || { tail -5 $O/bench_C_n2.err; exit 3; }
tail -c 300 $O/bench_C_n2.json
timeout -k 10 400 python -u bench.py --config D --gpus 2 --force-device 0 --dist-backend gloo --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/bench_D_n2.json 2> $O/bench_D_n2.err || { tail -5 $O/bench_D_n2.err; exit 4; }
tail -c 300 $O/bench_D_n2.json
