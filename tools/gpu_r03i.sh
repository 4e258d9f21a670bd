#!/bin/bash
# Round-3: rocprofv3 session (kernel trace + PMC passes) of config E.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03q}
O=gpurun_out/$T
mkdir -p $O
BENCH_ARGS="--config E" TAG=${T}_E OUT=$O/profe bash tools/profile_session.sh > $O/profe.log 2>&1 || { tail -20 $O/profe.log; exit 2; }
cp $O/profe/pmc_summary.json $O/pmc_e.json
echo done
