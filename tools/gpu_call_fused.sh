# GPU session: parity tests on the fused kernel, then interleaved A/B (legacy vs fused) on configs C and D.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== gpu tests (fused default)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_fused.log 2>&1; rc=$?
tail -25 gpurun_out/gpu_tests_fused.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== A/B C"
timeout -k 10 300 python tools/ab_match.py --rounds 5 --steps 10 --fast-g 2 --fused 0,1 --unroll 4,8 > gpurun_out/ab_fused_c.json 2> gpurun_out/ab_fused_c.err || { tail -20 gpurun_out/ab_fused_c.err; exit 3; }
cat gpurun_out/ab_fused_c.json
echo "== A/B D"
timeout -k 10 400 python tools/ab_match.py --config D --rounds 3 --steps 5 --fast-g 2 --fused 0,1 --unroll 4,8 > gpurun_out/ab_fused_d.json 2> gpurun_out/ab_fused_d.err || { tail -20 gpurun_out/ab_fused_d.err; exit 4; }
cat gpurun_out/ab_fused_d.json
