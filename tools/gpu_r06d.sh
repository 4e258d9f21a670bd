set -o pipefail
mkdir -p gpurun_out/r06d
for i in 1 2; do
VMQGB_RECLAIM=0 timeout -k 10 200 tools/bin/nif_harness 3 churn > gpurun_out/r06d/harness_noreclaim_$i.jsonl 2>> gpurun_out/r06d/err.txt || exit 1
timeout -k 10 200 tools/bin/nif_harness 3 churn > gpurun_out/r06d/harness_reclaim_$i.jsonl 2>> gpurun_out/r06d/err.txt || exit 1
done
echo done
