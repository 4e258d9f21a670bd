# GPU session: ACL parity tests, AC bench line, rocprofv3 kernel stats +
# PMC passes of the AC bench (tools/profile_session.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== acl gpu tests"
timeout -k 10 300 python -u -m pytest tests/test_acl.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_acl.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_acl.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== bench AC"
timeout -k 10 300 python bench.py --config AC --steps 20 --warmup 3 > gpurun_out/bench_ac.json 2> gpurun_out/bench_ac.err || { tail -20 gpurun_out/bench_ac.err; exit 3; }
cat gpurun_out/bench_ac.json
if [ -n "$PROFILE" ]; then
echo "== profile AC"
OUT=gpurun_out/prof_ac TAG=${TAG:-ac} BENCH_ARGS="--config AC" bash tools/profile_session.sh > gpurun_out/prof_ac.log 2>&1 || { tail -30 gpurun_out/prof_ac.log; exit 4; }
tail -3 gpurun_out/prof_ac.log
fi
