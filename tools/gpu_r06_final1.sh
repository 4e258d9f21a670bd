#!/bin/bash
# Round 6, final session 1 (frozen build): smoke, C's PMC session (kernel
# trace + FETCH / WRITE / L2 / LDS passes) and C's bench line.
set -o pipefail
O=gpurun_out/r06f1
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 4; }
tail -2 $O/smoke.log
OUT=$O/prof_C TAG=r06_C timeout -k 10 700 bash tools/profile_session.sh > $O/prof_C.log 2>&1 || { tail -5 $O/prof_C.log; exit 5; }
cp $O/prof_C/pmc_summary.json profiles/pmc_latest.json
timeout -k 10 400 python -u bench.py > $O/bench_C.json 2> $O/bench_C.err || { tail -5 $O/bench_C.err; exit 6; }
cat $O/bench_C.json
