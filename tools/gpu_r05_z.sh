#!/bin/bash
# Round 5, session z: C's and D's lines again on the final build (bench.py
# now reports the physical roofline fraction for both; library unchanged).
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_C.json 2> $O/bench_C.err || { tail -5 $O/bench_C.err; exit 3; }
tail -c 400 $O/bench_C.json
timeout -k 10 600 python -u bench.py --config D > $O/bench_D.json 2> $O/bench_D.err || { tail -5 $O/bench_D.err; exit 4; }
tail -c 400 $O/bench_D.json
