#!/bin/bash
# Round-3 session: config E at full size (50M subscriptions) on the library
# defaults, with its oracle sample and CPU baseline; then a kernel trace and
# the FETCH_SIZE / WRITE_SIZE passes of E (pmc_e.json).
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03e}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python3 -u bench.py --config E > $O/bench_E.json 2> $O/bench_E.err || { tail -20 $O/bench_E.err; exit 2; }
cat $O/bench_E.json
timeout -k 10 500 python3 -u bench.py --config D --no-cpu-baseline > $O/bench_D.json 2> $O/bench_D.err || { tail -20 $O/bench_D.err; exit 3; }
cat $O/bench_D.json
