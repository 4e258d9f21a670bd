set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r06c/tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r06c/tests.log
tail -3 gpurun_out/r06c/tests.log
VMQGB_REPLICAS=1 timeout -k 10 240 tools/bin/nif_harness 3 churn > gpurun_out/r06c/harness_rep1.jsonl 2> gpurun_out/r06c/harness_rep1.err && \
timeout -k 10 240 tools/bin/nif_harness 3 scale churn > gpurun_out/r06c/harness_rep0.jsonl 2> gpurun_out/r06c/harness_rep0.err
echo "harness rc=$?"
