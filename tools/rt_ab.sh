# A/B of retained-walk variants (build/ab/*.so from tools/build_variants.py):
# walk time on the full RT batch and on the heavy filters alone.
set -o pipefail
for so in build/ab/lib_*.so; do
  for cfg in "16 262144" "16 16" "0 262144"; do
    set -- $cfg
    VMQG_LIB_PATH=$so timeout -k 10 120 python bench.py --config RT --steps 20 --warmup 3 --no-cpu-baseline --rt-heavy $1 --rt-filters $2 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', $1, $2, round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" || echo "$so $cfg FAILED"
  done
done
