# fused trie-less match with the deferred look-back: parity tests on it and
# on the immediate variant, then R1 A/B
# libraries: VMQG_AB_DIR=build/ab8 python tools/build_variants.py nodefer
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
K="trieless or one_record or r1_r2 or word_lists or exact_filter"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$K" > $O/tests_defer.log 2>&1 || { tail -30 $O/tests_defer.log; exit 1; }
tail -1 $O/tests_defer.log
VMQG_LIB_PATH=$PWD/build/ab8/lib_nodefer.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "$K" > $O/tests_nodefer.log 2>&1 || { tail -30 $O/tests_nodefer.log; exit 2; }
tail -1 $O/tests_nodefer.log
B="python bench.py --config R1 --r-n 4096000 --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B > $O/r1_defer.json 2>> $O/err.txt || exit 3
VMQG_LIB_PATH=$PWD/build/ab8/lib_nodefer.so timeout -k 10 200 $B > $O/r1_nodefer.json 2>> $O/err.txt || exit 4
timeout -k 10 200 $B --config R2 > $O/r2_defer.json 2>> $O/err.txt || exit 5
echo done
