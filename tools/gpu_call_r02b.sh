# Round-2 GPU call: every -m gpu test; emit / store A/B on C and D; config D
# bench (churn, CPU baseline).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
echo "== A/B C"
timeout -k 10 300 python3 tools/ab_match.py --config C --opt emit_lean=0,1 --opt nt_stores=0,1 > gpurun_out/ab_c_emit.json 2> gpurun_out/ab_c_emit.err || { tail -20 gpurun_out/ab_c_emit.err; exit 2; }
cat gpurun_out/ab_c_emit.json
echo "== A/B D"
timeout -k 10 400 python3 tools/ab_match.py --config D --rounds 4 --opt emit_lean=0,1 > gpurun_out/ab_d_emit.json 2> gpurun_out/ab_d_emit.err || { tail -20 gpurun_out/ab_d_emit.err; exit 3; }
cat gpurun_out/ab_d_emit.json
echo "== config D"
timeout -k 10 600 python3 bench.py --config D --steps 10 --warmup 2 > gpurun_out/bench_D_${TAG}.json 2> gpurun_out/bench_D_${TAG}.err || { tail -30 gpurun_out/bench_D_${TAG}.err; exit 4; }
cat gpurun_out/bench_D_${TAG}.json
