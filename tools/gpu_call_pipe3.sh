#!/bin/bash
# EMIT copy with every load of a round issued before any store: parity + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_pipeline.py tests/test_gpu_parity.py > gpurun_out/pipe3_tests.log 2>&1 || { tail -30 gpurun_out/pipe3_tests.log; exit 1; }
tail -2 gpurun_out/pipe3_tests.log
timeout -k 10 400 python -u tools/ab_match.py --config C --rounds 4 --steps 10 --opt pipe=0,1 --opt mixed_bpc=4,8,16 > gpurun_out/ab_pipe3_c.json 2> gpurun_out/ab_pipe3_c.err || { tail -20 gpurun_out/ab_pipe3_c.err; exit 1; }
cat gpurun_out/ab_pipe3_c.json
