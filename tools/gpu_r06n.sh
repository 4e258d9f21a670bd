# config A: fixed-cost knobs swept on one load
set -o pipefail
mkdir -p gpurun_out/r06n
timeout -k 10 300 python -u tools/opt_sweep.py --config A --steps 50 "dedupe=0" "dedupe=1" "dedupe=2,fast_g=1" "fast_g=2" "fast_g=4" "fast_g=0,count_bpc=8" "count_bpc=3" "count_bpc=5,emit_bpc=8" "emit_bpc=32" "emit_bpc=16,dd_g=1" "dd_g=2" "dd_g=4" > gpurun_out/r06n/a_sweep.jsonl 2> gpurun_out/r06n/a_sweep.err || exit 1
echo done
