#!/bin/bash
# Round 5, session p: heavy_min 512 on D and E (interleaved in one process each).
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 400 python -u tools/ab_match.py --config D --rounds 4 --opt heavy_min=0,512,1024 > $O/ab_D_heavy.json 2> $O/ab_D.err || { tail -5 $O/ab_D.err; exit 4; }
cat $O/ab_D_heavy.json
timeout -k 10 600 python -u tools/ab_match.py --config E --e-scale 1.0 --rounds 4 --opt heavy_min=0,512 > $O/ab_E_heavy.json 2> $O/ab_E.err || { tail -5 $O/ab_E.err; exit 5; }
cat $O/ab_E_heavy.json
