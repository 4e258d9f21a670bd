# R1: the fused match with the next tile's ticket and publishes fetched while
# the previous tile's entries are written (out of tree: profiles/ab_r06_fused/r06x_prefetch.diff applied, built to build/ab9/lib_pf.so),
# parity tests on it, then against the shipped build
set -o pipefail
O=gpurun_out/r06x
mkdir -p $O
VMQG_LIB_PATH=$PWD/build/ab9/lib_pf.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "trieless or one_record or r1_r2 or word_lists or exact_filter" > $O/tests_pf.log 2>&1 || { tail -30 $O/tests_pf.log; exit 1; }
tail -1 $O/tests_pf.log
B="python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B > $O/r1_shipped.json 2>> $O/err.txt || exit 3
VMQG_LIB_PATH=$PWD/build/ab9/lib_pf.so timeout -k 10 200 $B > $O/r1_pf.json 2>> $O/err.txt || exit 4
VMQG_LIB_PATH=$PWD/build/ab9/lib_pf.so timeout -k 10 200 $B --config R2 > $O/r2_pf.json 2>> $O/err.txt || exit 5
echo done
