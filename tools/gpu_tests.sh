# Every -m gpu test on the box (one pytest process), log under gpurun_out/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${T:-900} python -u -m pytest tests -m gpu ${SEL:-} --maxfail=${MAXFAIL:-6} -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -40 gpurun_out/gpu_tests.log
echo "pytest rc=$rc"
exit $rc
