# RT walk diagnostics: retain parity tests, then the walk time with and
# without the heavy filters, at full and tiny batch size.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_retain.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_retain.log 2>&1 || { tail -30 gpurun_out/gpu_retain.log; exit 1; }
tail -1 gpurun_out/gpu_retain.log
for h in 0 16; do for nf in 262144 16; do
timeout -k 10 120 python bench.py --config RT --steps 20 --warmup 3 --no-cpu-baseline --rt-heavy $h --rt-filters $nf 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($h, $nf, d['ms_per_step'], d['kernel_us'])" || exit 1
done; done
