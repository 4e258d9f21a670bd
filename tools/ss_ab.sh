# A/B of shared-subscription select variants (build/ab/*.so from
# tools/build_variants.py): select kernel time on the SS batch.
set -o pipefail
for so in build/ab/lib_*.so; do
  VMQG_LIB_PATH=$so timeout -k 10 150 python bench.py --config SS --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', round(d['ms_per_step']*1e3,1), d['kernel_us'])" || { echo "$so FAILED"; exit 1; }
done
