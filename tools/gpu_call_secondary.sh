#!/bin/bash
# secondary bench lines on the current build: D (churn), SS, RT, AC, then B
set -o pipefail
mkdir -p gpurun_out/sec
for c in D SS RT AC B; do
  echo "== $c"
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/sec/bench_$c.json 2> gpurun_out/sec/bench_$c.err || { tail -20 gpurun_out/sec/bench_$c.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sec/bench_$c.json')); r=d.get('roofline') or {}; print('$c', '%.3g'%d['value'], d['unit'], 'frac', r.get('frac'))"
done
