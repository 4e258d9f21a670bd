#!/bin/bash
# Round-3 session: rocprofv3 sessions (kernel trace + PMC passes) of
# configs C and D on the current build, copied to gpurun_out/<tag>/pmc_{c,d}.json.
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03g}
O=gpurun_out/$T
mkdir -p $O
TAG=${T}_C OUT=$O/profc bash tools/profile_session.sh > $O/profc.log 2>&1 || { tail -20 $O/profc.log; exit 2; }
cp $O/profc/pmc_summary.json $O/pmc_c.json
BENCH_ARGS="--config D" TAG=${T}_D OUT=$O/profd bash tools/profile_session.sh > $O/profd.log 2>&1 || { tail -20 $O/profd.log; exit 3; }
cp $O/profd/pmc_summary.json $O/pmc_d.json
echo done
