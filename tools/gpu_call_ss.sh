# Shared-subscription dispatcher on one GPU: its GPU tests, then the SS bench
# line (config D match output, prefer_local) with the CPU baseline.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== shared gpu tests"
timeout -k 10 400 python -u -m pytest tests/test_shared.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ss_tests.log 2>&1; rc=$?
tail -15 gpurun_out/ss_tests.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then grep -B5 -A30 "Error\|FAILED" gpurun_out/ss_tests.log | head -80; exit $rc; fi
echo "== bench SS"
timeout -k 10 500 python bench.py --config SS ${SS_ARGS:-} > gpurun_out/bench_ss.json 2> gpurun_out/bench_ss.err || { tail -20 gpurun_out/bench_ss.err; exit 3; }
cat gpurun_out/bench_ss.json
tail -5 gpurun_out/bench_ss.err
