# Secondary bench lines (configs D, E, A, B, R1, R2) + the N=2 rehearsal of
# the replication path (gloo, both ranks on the one GPU).  Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
for c in D E A B R1 R2; do
  echo "== bench $c"
  timeout -k 10 500 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err
  rc=$?; tail -2 gpurun_out/bench_$c.err; cat gpurun_out/bench_$c.json; echo "rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
echo "== N=2 rehearsal (gloo, one GPU)"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --dist-backend gloo --force-device 0 --no-cpu-baseline > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
rc=$?; tail -4 gpurun_out/bench_n2.err; cat gpurun_out/bench_n2.json; echo "n2 rc=$rc"
exit $rc
