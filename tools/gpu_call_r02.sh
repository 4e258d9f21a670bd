set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
echo "== store ceiling"
timeout -k 10 120 ./tools/bin/store_ceiling > gpurun_out/store_ceiling.json 2>&1 || { cat gpurun_out/store_ceiling.json; exit 2; }
cat gpurun_out/store_ceiling.json
TAG=r02_v2 NOPROF=1 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_bench_prof.sh
