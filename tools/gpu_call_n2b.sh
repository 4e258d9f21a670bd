# N=2 replica bisect: the GPU dist tests, then config D at 0.1 scale, two
# ranks on one card (gloo), under the default build and two kernel variants.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dist.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/n2_dist_tests.log 2>&1; echo "dist tests rc=$?"; tail -5 $O/n2_dist_tests.log
for v in default; do
  unset VMQG_LIB_PATH; [ $v != default ] && export VMQG_LIB_PATH=build/ab/lib_$v.so
  echo "== D N=2 $v"
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --config D --dist-backend gloo --force-device 0 --d-scale 0.1 --steps 3 --warmup 1 --no-cpu-baseline > $O/d_n2_$v.json 2> $O/d_n2_$v.err; echo "rc=$?"
  grep -h "RuntimeError\|replicated" $O/d_n2_$v.err | head -4
done
