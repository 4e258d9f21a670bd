# GPU session: N=2 rehearsal on one card (gloo), config D kernel trace, config E bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_d
echo "== N=2 rehearsal (gloo, both ranks on device 0)"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --force-device 0 \
  --no-cpu-baseline > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { tail -30 gpurun_out/bench_n2.err; exit 3; }
cat gpurun_out/bench_n2.json
echo "== config D kernel trace"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d -o run --output-format csv -- \
  python3 bench.py --config D --steps 3 --warmup 1 > gpurun_out/prof_d/log.txt 2>&1 || { tail -30 gpurun_out/prof_d/log.txt; exit 4; }
tail -3 gpurun_out/prof_d/log.txt
echo "== config E (scale ${E_SCALE:-0.2})"
timeout -k 10 600 python bench.py --config E --e-scale ${E_SCALE:-0.2} --steps 10 --warmup 2 > gpurun_out/bench_e.json 2> gpurun_out/bench_e.err || { tail -30 gpurun_out/bench_e.err; exit 5; }
tail -3 gpurun_out/bench_e.err; cat gpurun_out/bench_e.json
