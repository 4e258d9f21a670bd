#!/bin/bash
# one lane per publish in the fast tier (fast_g=1; EMIT without walk lists):
# parity, then A/B on C, D and E (0.2)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py -k "deferral_heavy or golden or churn" > gpurun_out/g1_tests.log 2>&1 || { tail -30 gpurun_out/g1_tests.log; exit 1; }
tail -1 gpurun_out/g1_tests.log
for c in C D E; do
  timeout -k 10 500 python -u tools/ab_match.py --config $c --rounds 4 --steps 8 --d-scale 0.5 --opt fast_g=1,2 > gpurun_out/ab_g1_$c.json 2> gpurun_out/ab_g1_$c.err || { tail -20 gpurun_out/ab_g1_$c.err; exit 2; }
  cat gpurun_out/ab_g1_$c.json
done
