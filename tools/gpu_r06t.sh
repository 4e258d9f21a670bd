# R1: the deferred-look-back fused match, tile-shape variants
# libraries: VMQG_AB_DIR=build/ab8 python tools/build_variants.py k2 k1bpc6 k1bpc8 k2bpc5 k2bpc6 k3 bpc8
set -o pipefail
O=gpurun_out/r06t2
mkdir -p $O
B="python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B > $O/r1_default.json 2>> $O/err.txt || exit 3
for v in k2 k1bpc6 k1bpc8 k2bpc5; do
VMQG_LIB_PATH=$PWD/build/ab8/lib_$v.so timeout -k 10 200 $B > $O/r1_$v.json 2>> $O/err.txt || exit 4
done
echo done
