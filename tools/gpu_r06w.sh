# R1: the fused match at occupancy 5 / 6 (VGPR cap, small spills) against the same source uncapped
# libraries: build/ab9 (the waves-per-EU cap patched in out of tree: VMQG_FX_WPE)
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
B="python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e"
for v in base wpe5bpc5 k1wpe6bpc6; do
VMQG_LIB_PATH=$PWD/build/ab9/lib_$v.so timeout -k 10 200 $B > $O/r1_$v.json 2>> $O/err.txt || exit 4
done
echo done
