# config E: EMIT / COUNT grid and lane knobs swept on one load
set -o pipefail
mkdir -p gpurun_out/r06m
timeout -k 10 600 python -u tools/opt_sweep.py --config E "emit_bpc=8" "emit_bpc=32" "emit_bpc=0" "emit_bpc=16,fast_g=2" "fast_g=4" "fast_g=1" "fast_g=0,count_bpc=8" "count_bpc=3" "count_bpc=5,dd_g=1" "dd_g=4,heavy_min=256" "heavy_min=0" > gpurun_out/r06m/e_sweep.jsonl 2> gpurun_out/r06m/e_sweep.err || exit 1
echo done
