# The whole -m gpu suite as the driver runs it (E now at full size), with
# per-test durations; a heartbeat file shows progress through long tests.
set -o pipefail
mkdir -p gpurun_out/r06h
( while sleep 50; do date +%s >> gpurun_out/r06h/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --durations=40 > gpurun_out/r06h/tests.log 2>&1
rc=$?
kill $HB
echo "tests rc=$rc" >> gpurun_out/r06h/tests.log
exit $rc
