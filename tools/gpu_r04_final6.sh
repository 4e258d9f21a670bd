#!/bin/bash
# Round 4 final build, call 6: two ranks on the one GPU (gloo control and
# data group) rehearsing the N>1 bench paths of C and D; the driver's real
# N>1 runs use RCCL on separate GPUs.
set -o pipefail
O=gpurun_out/final6
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 10 --warmup 2 --force-device 0 --dist-backend gloo --no-cpu-baseline > $O/bench_C_n2.json 2> $O/bench_C_n2.err &&
timeout -k 10 420 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --config D --gpus 2 --steps 3 --warmup 1 --force-device 0 --dist-backend gloo --no-cpu-baseline > $O/bench_D_n2.json 2> $O/bench_D_n2.err
