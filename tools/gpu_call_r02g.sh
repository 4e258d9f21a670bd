# Restored-tree re-run: every -m gpu test, smoke, the default bench line, and
# the rocprof session (kernel trace + PMC passes) on this exact build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
T=700 bash tools/gpu_tests.sh || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
cat $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
cat $O/bench.json
TAG=${TAG:-r02_v10} bash tools/profile_session.sh || exit 4
