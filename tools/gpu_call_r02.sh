# Round-2 GPU call: all -m gpu tests, then the default bench (config C) and
# config D, without profiling.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
TAG=${TAG:-r02} NOPROF=1 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_bench_prof.sh || exit 3
echo "== config D"
timeout -k 10 500 python3 bench.py --config D --steps 10 --warmup 2 > gpurun_out/bench_D_${TAG:-r02}.json 2> gpurun_out/bench_D_${TAG:-r02}.err || { tail -30 gpurun_out/bench_D_${TAG:-r02}.err; exit 4; }
cat gpurun_out/bench_D_${TAG:-r02}.json
