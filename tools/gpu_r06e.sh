set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "trieless or r1_r2 or golden or churn_fold or mountpoints_are" > gpurun_out/r06e/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/r06e/tests.log; tail -3 gpurun_out/r06e/tests.log
[ $rc -eq 0 ] || exit 1
for f in 1 0; do
timeout -k 10 300 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e --vmqg-opt fused=$f > gpurun_out/r06e/r1_fused$f.json 2> gpurun_out/r06e/r1_fused$f.err || exit 2
done
echo done
