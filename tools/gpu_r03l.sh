#!/bin/bash
# Round-3 final lines: the default bench (config C, as the driver runs it:
# CPU baseline and end-to-end included), config D, and the NIF harness.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03u}
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench_C.json 2> $O/bench_C.err || { tail -5 $O/bench_C.err; exit 2; }
cat $O/bench_C.json
timeout -k 10 500 python3 bench.py --config D > $O/bench_D.json 2> $O/bench_D.err || { tail -5 $O/bench_D.err; exit 3; }
cat $O/bench_D.json
timeout -k 10 400 tools/bin/nif_harness 2 > $O/nif.jsonl 2> $O/nif.err || { tail -5 $O/nif.err; exit 4; }
cat $O/nif.jsonl
echo done
