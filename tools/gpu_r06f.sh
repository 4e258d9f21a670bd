set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 200 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e > gpurun_out/r06f/r1_default.json 2> gpurun_out/r06f/err.txt || exit 2
for v in exact2x fxk2 fxk8 fxbpc8 fxk2bpc8; do
VMQG_LIB_PATH=$PWD/build/ab6/lib_$v.so timeout -k 10 200 python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e > gpurun_out/r06f/r1_$v.json 2>> gpurun_out/r06f/err.txt || exit 3
done
echo done
