#!/bin/bash
# Round 5, session b: smoke; C's line on the new exact-slot build; the
# launcher-less 2-rank rehearsal (--gpus 2 on one GPU, gloo); R1 at the
# reference suite's 4,096,000; A at fast_g 1 / 2 / 4; the retained / ACL /
# vmq_reg NIF glue GPU tests; a LITE rocprofv3 session of R1.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_C.json 2> $O/bench_C.err &&
timeout -k 10 300 python -u bench.py --gpus 2 --force-device 0 --dist-backend gloo --no-cpu-baseline > $O/bench_C_n2.json 2> $O/bench_C_n2.err &&
timeout -k 10 300 python -u bench.py --config R1 --r-n 4096000 > $O/bench_R1.json 2> $O/bench_R1.err &&
for g in 1 2 4; do
  timeout -k 10 200 python -u bench.py --config A --fast-g $g --no-cpu-baseline > $O/bench_A_g$g.json 2> $O/bench_A_g$g.err || exit 5
done &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_nif_layer.py -m gpu > $O/nif_tests.log 2>&1 &&
LITE=1 OUT=$O/prof_R1 BENCH_ARGS="--config R1 --r-n 4096000" TAG=r05_R1 timeout -k 10 600 bash tools/profile_session.sh > $O/prof_R1.log 2>&1
rc=$?
tail -3 $O/nif_tests.log
exit $rc
