# GPU session: retained-store parity tests, RT bench line, rocprofv3 kernel
# stats + PMC passes of the RT bench (tools/profile_session.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== retain gpu tests"
timeout -k 10 400 python -u -m pytest tests/test_retain.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_retain.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_retain.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== bench RT"
timeout -k 10 300 python bench.py --config RT --steps 20 --warmup 3 > gpurun_out/bench_rt.json 2> gpurun_out/bench_rt.err || { tail -20 gpurun_out/bench_rt.err; exit 3; }
cat gpurun_out/bench_rt.json
echo "== profile RT"
OUT=gpurun_out/prof_rt TAG=${TAG:-rt} BENCH_ARGS="--config RT" bash tools/profile_session.sh > gpurun_out/prof_rt.log 2>&1 || { tail -30 gpurun_out/prof_rt.log; exit 4; }
tail -3 gpurun_out/prof_rt.log
