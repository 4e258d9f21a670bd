#!/bin/bash
# Round-3 re-entry check: the whole GPU suite and smoke() on the rebuilt
# library, then the default bench line (as the driver runs it).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r03m}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 2; }
tail -3 $O/tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 240 python3 bench.py > $O/bench_C.json 2> $O/bench_C.err || { tail -5 $O/bench_C.err; exit 4; }
cat $O/bench_C.json
echo done
