# R1 fused match with the one-record exact slots: trie-less parity tests, then
# the shipped default against exact_one=0 and the tile-shape variants (build/ab6)
set -o pipefail
mkdir -p gpurun_out/r06g
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "trieless or exact or word_lists or reclaim or one_record" > gpurun_out/r06g/tests.log 2>&1 || exit 1
B="python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B > gpurun_out/r06g/r1_default.json 2> gpurun_out/r06g/err.txt || exit 2
timeout -k 10 200 $B --vmqg-opt exact_one=0 > gpurun_out/r06g/r1_noone.json 2>> gpurun_out/r06g/err.txt || exit 3
for v in fxk2 fxk3 fxk2u2 fxk2u2bpc5 fxk2bpc8; do
VMQG_LIB_PATH=$PWD/build/ab6/lib_$v.so timeout -k 10 200 $B > gpurun_out/r06g/r1_$v.json 2>> gpurun_out/r06g/err.txt || exit 4
done
echo done
