# GPU session: retained-store parity tests, match parity subset, bench C.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== retain gpu tests"
timeout -k 10 400 python -u -m pytest tests/test_retain.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_retain.log 2>&1; rc=$?
tail -30 gpurun_out/gpu_retain.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== match gpu tests"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== bench C"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 3; }
cat gpurun_out/bench.json
