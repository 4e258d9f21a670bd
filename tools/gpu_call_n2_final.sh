#!/bin/bash
# N=2 rehearsals on the one card (gloo, both ranks on device 0) of the final
# build: config C, then config D at 0.1 scale (image + patch broadcast,
# replica parity)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
echo "== C N=2 rehearsal"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --dist-backend gloo --force-device 0 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $O/c_n2.json 2> $O/c_n2.err || { tail -30 $O/c_n2.err; exit 8; }
cat $O/c_n2.json
echo "== D N=2 rehearsal"
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --config D --dist-backend gloo --force-device 0 --d-scale 0.1 --steps 5 --warmup 1 --no-cpu-baseline > $O/d_n2.json 2> $O/d_n2.err || { tail -30 $O/d_n2.err; exit 7; }
cat $O/d_n2.json
