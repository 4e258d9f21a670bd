#!/bin/bash
# Round 5, session j: heavy-publish routing by XCD on E and D (interleaved
# A/B in one process), A's lanes per publish, A's output shape.
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 200 python -u tools/diag_shape.py A > $O/diag_A.txt 2>&1 || { tail -5 $O/diag_A.txt; exit 3; }
cat $O/diag_A.txt
timeout -k 10 200 python -u tools/ab_match.py --config A --opt fast_g=1,2,4 > $O/ab_A_fastg.json 2> $O/ab_A.err || { tail -5 $O/ab_A.err; exit 4; }
cat $O/ab_A_fastg.json
timeout -k 10 400 python -u tools/ab_match.py --config D --rounds 4 --opt heavy_min=0,256,128 > $O/ab_D_heavy.json 2> $O/ab_D.err || { tail -5 $O/ab_D.err; exit 5; }
cat $O/ab_D_heavy.json
timeout -k 10 600 python -u tools/ab_match.py --config E --e-scale 1.0 --rounds 4 --opt heavy_min=0,256,128,64 > $O/ab_E_heavy.json 2> $O/ab_E.err || { tail -5 $O/ab_E.err; exit 6; }
cat $O/ab_E_heavy.json
