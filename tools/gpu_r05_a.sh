set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_word_lists.py tests/test_gpu_parity.py -m gpu > gpurun_out/r05a_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r05a_tests.log
exit $rc
