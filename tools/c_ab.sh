# Headline (config C) under each build/ab/*.so variant (tools/build_variants.py),
# twice, interleaved; then the default bench line with the end-to-end figure.
set -o pipefail
for rep in 1 2; do
for so in build/ab/lib_*.so; do
  VMQG_LIB_PATH=$so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $so)', round(d['ms_per_step']*1e3,1), {k: round(v,1) for k,v in d['kernel_us'].items()})" || echo "$so FAILED"
done
done
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err || { tail -20 gpurun_out/bench_e2e.err; exit 3; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_e2e.json')); print(d['value'], d['end_to_end'])"
