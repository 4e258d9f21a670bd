# R1: the fused kernel with more 64-publish chunks per wave (fewer waves)
set -o pipefail
mkdir -p gpurun_out/r06i
B="python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B > gpurun_out/r06i/r1_default.json 2> gpurun_out/r06i/err.txt || exit 2
for v in fxk6 fxk8; do
VMQG_LIB_PATH=$PWD/build/ab6/lib_$v.so timeout -k 10 200 $B > gpurun_out/r06i/r1_$v.json 2>> gpurun_out/r06i/err.txt || exit 4
done
echo done
