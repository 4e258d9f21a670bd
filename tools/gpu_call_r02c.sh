# Round-2 GPU call: grid-cap A/B on C, config D churn line, config E at full
# size (50M subscriptions).
set -o pipefail
mkdir -p gpurun_out
echo "== A/B C grid caps"
timeout -k 10 300 python3 tools/ab_match.py --config C --rounds 5 --opt count_bpc=4,8,16 --opt emit_bpc=4,8,16 > gpurun_out/ab_c_bpc.json 2> gpurun_out/ab_c_bpc.err || { tail -20 gpurun_out/ab_c_bpc.err; exit 2; }
cat gpurun_out/ab_c_bpc.json
echo "== config D"
timeout -k 10 400 python3 bench.py --config D --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_D_${TAG}.json 2> gpurun_out/bench_D_${TAG}.err || { tail -30 gpurun_out/bench_D_${TAG}.err; exit 4; }
cat gpurun_out/bench_D_${TAG}.json
echo "== config E (50M)"
timeout -k 10 900 python3 -u bench.py --config E --steps 10 --warmup 2 > gpurun_out/bench_E_${TAG}.json 2> gpurun_out/bench_E_${TAG}.err || { tail -30 gpurun_out/bench_E_${TAG}.err; exit 5; }
cat gpurun_out/bench_E_${TAG}.json
tail -5 gpurun_out/bench_E_${TAG}.err
