#!/bin/bash
# pipelined match v2 (static striding): parity, then A/B pipe x mixed_bpc
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_pipeline.py > gpurun_out/pipe2_tests.log 2>&1 || { tail -30 gpurun_out/pipe2_tests.log; exit 1; }
tail -2 gpurun_out/pipe2_tests.log
timeout -k 10 400 python -u tools/ab_match.py --config C --rounds 4 --steps 10 --opt pipe=0,1 --opt mixed_bpc=4,8,16 > gpurun_out/ab_pipe_c.json 2> gpurun_out/ab_pipe_c.err || { tail -20 gpurun_out/ab_pipe_c.err; exit 1; }
cat gpurun_out/ab_pipe_c.json
