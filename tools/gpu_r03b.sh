#!/bin/bash
# Round-3 session after the hang fix: fusion-option matrix on the
# deferral-heavy scenario (stops at the first failure), the whole -m gpu
# suite, bench lines of C and D, the NIF harness.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03d}
mkdir -p $O
VMQG_DEBUG_SYNC=15 timeout -k 10 200 python3 -u tools/dbg_defer.py > $O/defer.log 2>&1 || { grep -v "debug: .* done" $O/defer.log | tail -20; exit 2; }
grep -v "debug: .* done" $O/defer.log
timeout -k 10 900 python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_C.json 2> $O/bench_C.err || { tail -5 $O/bench_C.err; exit 6; }
cat $O/bench_C.json
timeout -k 10 500 python3 bench.py --config D --no-cpu-baseline > $O/bench_D.json 2> $O/bench_D.err || { tail -5 $O/bench_D.err; exit 7; }
cat $O/bench_D.json
timeout -k 10 400 tools/bin/nif_harness 2 > $O/nif.jsonl 2> $O/nif.err || { tail -5 $O/nif.err; exit 8; }
cat $O/nif.jsonl
echo done
