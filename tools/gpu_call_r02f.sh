# Every -m gpu test on this build, then the N=2 rehearsals (gloo, both ranks
# on the one card): config D at 0.1 scale with replica image checks, config C.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
T=700 bash tools/gpu_tests.sh || exit 1
echo "== D N=2"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --config D --dist-backend gloo --force-device 0 --d-scale 0.1 --steps 5 --warmup 1 --no-cpu-baseline > $O/d_n2.json 2> $O/d_n2.err || { grep -h "RuntimeError\|regions" $O/d_n2.err | head; exit 7; }
cat $O/d_n2.json
echo "== C N=2"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --dist-backend gloo --force-device 0 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/c_n2.json 2> $O/c_n2.err || { tail -20 $O/c_n2.err; exit 8; }
cat $O/c_n2.json
