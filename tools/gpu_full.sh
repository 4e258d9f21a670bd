# Round-end rehearsal on one GPU: every -m gpu test, smoke(), the default
# bench line (config C + CPU baseline), and the N=2 path (gloo, both ranks
# on device 0).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_all.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then tail -40 gpurun_out/gpu_all.log; exit $rc; fi
echo "== smoke"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 5; }
tail -1 gpurun_out/smoke.log
echo "== bench (default)"
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 3; }
cat gpurun_out/bench.json
echo "== bench N=2 rehearsal"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --force-device 0 --no-cpu-baseline > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { tail -20 gpurun_out/bench_n2.err; exit 4; }
cat gpurun_out/bench_n2.json
