#!/bin/bash
# Round 5, session t: D's line again (its host-apply figure fixed in
# bench.py; the library is the final build), then R1's exact-table load
# A/B through the size hint (load 0.49 / 0.24 / 0.12; no library change).
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 600 python -u bench.py --config D > $O/bench_D.json 2> $O/bench_D.err || { tail -5 $O/bench_D.err; exit 3; }
tail -c 300 $O/bench_D.json
for m in 1 2 4 1; do
  timeout -k 10 240 python -u bench.py --config R1 --r-n 4096000 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --exact-hint-mult $m > $O/b_R1_m$m.json 2> $O/b_R1_m$m.err || { tail -5 $O/b_R1_m$m.err; exit 4; }
  python3 -c "import json; d=json.load(open('$O/b_R1_m$m.json')); print('R1 mult $m', '%.4g' % d['value'], d['arena_bytes'], {k: round(v,1) for k,v in d['kernel_us'].items()})" | tee -a $O/ab.txt
done
# N = 2 without a launcher: bench.py spawns both ranks (this box has one GPU: both on device 0, gloo)
timeout -k 10 300 python -u bench.py --gpus 2 --force-device 0 --dist-backend gloo --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/bench_C_n2.json 2> $O/bench_C_n2.err || { tail -5 $O/bench_C_n2.err; exit 5; }
tail -c 300 $O/bench_C_n2.json
