# retain parity tests on the default build, then the A/B variants
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_retain.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_retain.log 2>&1 || { tail -30 gpurun_out/gpu_retain.log; exit 1; }
tail -1 gpurun_out/gpu_retain.log
bash tools/rt_ab.sh
