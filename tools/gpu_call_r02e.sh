# Round-2 GPU call: the headline bench + rocprof session of this build, and a
# COUNT occupancy A/B (4 vs 5 waves/SIMD builds, alternating processes).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "config_c or golden or churn" > gpurun_out/gpu_quick.log 2>&1 || { tail -30 gpurun_out/gpu_quick.log; exit 1; }
tail -2 gpurun_out/gpu_quick.log
TAG=${TAG} bash tools/gpu_bench_prof.sh || exit 3
echo "== A/B COUNT waves per SIMD"
for i in 1 2; do
  for v in default count_wpe5; do
    VMQG_LIB_PATH=build/ab/lib_$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-e2e > gpurun_out/ab_wpe_${v}_$i.json 2>/dev/null || exit 5
    python3 -c "import json; d=json.load(open('gpurun_out/ab_wpe_${v}_$i.json')); print('$v', d['ms_per_step'], d['kernel_us'])"
  done
done
