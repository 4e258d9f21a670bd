# GPU session: fused-kernel parity subset, then interleaved A/B on configs C and D.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== gpu tests (subset)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "${TESTS_K:-config_full_parity or wide_frontier or churn_fold or config_d}" > gpurun_out/gpu_tests_sub.log 2>&1; rc=$?
tail -5 gpurun_out/gpu_tests_sub.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== A/B C"
timeout -k 10 300 python tools/ab_match.py --rounds 5 --steps 10 --fast-g 2 --fused 0,1 --unroll ${UNROLL:-4} > gpurun_out/ab_c.json 2> gpurun_out/ab_c.err || { tail -20 gpurun_out/ab_c.err; exit 3; }
cat gpurun_out/ab_c.json
if [ -n "$AB_D" ]; then
echo "== A/B D"
timeout -k 10 400 python tools/ab_match.py --config D --rounds 3 --steps 5 --fast-g 2 --fused 0,1 --unroll ${UNROLL:-4} > gpurun_out/ab_d.json 2> gpurun_out/ab_d.err || { tail -20 gpurun_out/ab_d.err; exit 4; }
cat gpurun_out/ab_d.json
fi
