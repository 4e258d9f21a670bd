#!/bin/bash
# Round 4 final build, call 5: R2's line again after the bench's roofline
# choice learned that the EMIT tail can dominate.
set -o pipefail
O=gpurun_out/final5
mkdir -p $O
timeout -k 10 300 python -u bench.py --config R2 --r-n 4096000 > $O/bench_R2.json 2> $O/bench_R2.err
