#!/bin/bash
# Round 4: interleaved A/Bs of batch dedupe and output groups (tools/ab_match.py).
set -o pipefail
mkdir -p gpurun_out/r04g
timeout -k 10 240 python -u tools/ab_match.py --config C --rounds 4 --opt dedupe=0,1 > gpurun_out/r04g/ab_C.json 2> gpurun_out/r04g/ab_C.err &&
timeout -k 10 300 python -u tools/ab_match.py --config E --rounds 4 --opt dedupe=0,1 > gpurun_out/r04g/ab_E02.json 2> gpurun_out/r04g/ab_E02.err &&
timeout -k 10 420 python -u tools/ab_match.py --config D --rounds 3 --opt dedupe=0,1 --opt groups=0,1 > gpurun_out/r04g/ab_D.json 2> gpurun_out/r04g/ab_D.err
