#!/bin/bash
# Round 5, session c: parity of the new exact layout + auto exbits filter
# (word lists, golden scenarios, churn, configs A/B, filter modes), then R1
# auto vs filter forced on, C and D on the auto default, R1's LITE profile.
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_word_lists.py \
  tests/test_gpu_parity.py -m gpu -k "word or golden or churn or config_full or exact_filter or cluster or frontier or dedupe" > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config R1 --r-n 4096000 --no-cpu-baseline > $O/bench_R1.json 2> $O/bench_R1.err &&
timeout -k 10 300 python -u bench.py --config R1 --r-n 4096000 --no-cpu-baseline --vmqg-opt exfilter=1 > $O/bench_R1_f1.json 2> $O/bench_R1_f1.err &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_C.json 2> $O/bench_C.err &&
timeout -k 10 420 python -u bench.py --config D --no-cpu-baseline > $O/bench_D.json 2> $O/bench_D.err &&
LITE=1 OUT=$O/prof_R1 BENCH_ARGS="--config R1 --r-n 4096000" TAG=r05_R1 timeout -k 10 600 bash tools/profile_session.sh > $O/prof_R1.log 2>&1
rc=$?
tail -3 $O/tests.log
exit $rc
