# Round-2 GPU call: every -m gpu test, the NIF host-half harness, config D.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
echo "== NIF harness"
timeout -k 10 400 ./tools/bin/nif_harness > gpurun_out/nif_harness_${TAG}.jsonl 2> gpurun_out/nif_harness_${TAG}.err || { tail -20 gpurun_out/nif_harness_${TAG}.err; exit 2; }
cat gpurun_out/nif_harness_${TAG}.jsonl
echo "== config D"
timeout -k 10 400 python3 bench.py --config D --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_D_${TAG}.json 2> gpurun_out/bench_D_${TAG}.err || { tail -30 gpurun_out/bench_D_${TAG}.err; exit 4; }
cat gpurun_out/bench_D_${TAG}.json
