#!/bin/bash
# Round-3 GPU session: new parity tests first, then the whole -m gpu suite,
# then bench lines of C, D and E (kernel timing of all five launches), and
# a rocprofv3 session (kernel trace + PMC passes) of config D.
# usage: bash tools/gpu_r03.sh <tag> <steps...>   steps: tests bench profd profc profe
set -o pipefail
export TMPDIR=/tmp
T=${1:-r03}; shift
O=gpurun_out/$T
mkdir -p $O
PYT="python -u -m pytest -x -v --durations=15 --timeout 300 --timeout-method thread"
for step in "$@"; do
  case $step in
  tests)
    timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_nif_layer.py -m gpu -k "many_key or one_record or config_d or config_e or deferral_heavy or retry or epoch or concurrent_batchers" > $O/tests_new.log 2>&1 || { tail -40 $O/tests_new.log; exit 2; }
    tail -1 $O/tests_new.log
    timeout -k 10 900 $PYT tests -m gpu > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
    tail -1 $O/tests.log ;;
  bench)
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e > $O/bench_C.json 2> $O/bench_C.err || { tail -20 $O/bench_C.err; exit 4; }
    cat $O/bench_C.json
    timeout -k 10 400 python3 bench.py --config D --no-cpu-baseline > $O/bench_D.json 2> $O/bench_D.err || { tail -20 $O/bench_D.err; exit 5; }
    cat $O/bench_D.json
    timeout -k 10 500 python3 bench.py --config E --no-cpu-baseline > $O/bench_E.json 2> $O/bench_E.err || { tail -20 $O/bench_E.err; exit 6; }
    cat $O/bench_E.json ;;
  profc)
    TAG=${T}_C OUT=$O/profc bash tools/profile_session.sh > $O/profc.log 2>&1 || { tail -20 $O/profc.log; exit 7; }
    cp $O/profc/pmc_summary.json $O/pmc_c.json ;;
  profd)
    BENCH_ARGS="--config D" TAG=${T}_D OUT=$O/profd bash tools/profile_session.sh > $O/profd.log 2>&1 || { tail -20 $O/profd.log; exit 8; }
    cp $O/profd/pmc_summary.json $O/pmc_d.json ;;
  profe)
    BENCH_ARGS="--config E --steps 5" TAG=${T}_E OUT=$O/profe bash tools/profile_session.sh > $O/profe.log 2>&1 || { tail -20 $O/profe.log; exit 9; }
    cp $O/profe/pmc_summary.json $O/pmc_e.json ;;
  nif)
    timeout -k 10 400 tools/bin/nif_harness 2 > $O/nif.jsonl 2> $O/nif.err || { tail -20 $O/nif.err; exit 10; }
    cat $O/nif.jsonl ;;
  esac
done
echo done
