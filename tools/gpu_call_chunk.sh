# Chunk-total offsets: every -m gpu test, then configs C and E (0.2 scale).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
T=700 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/chunk_C.json 2> $O/chunk_C.err || { tail -20 $O/chunk_C.err; exit 5; }
python3 -c "import json;d=json.load(open('$O/chunk_C.json'));print('C', d['value'], d.get('kernel_us'))"
timeout -k 10 300 python3 -u bench.py --config E --e-scale 0.2 --steps 10 --warmup 2 --no-cpu-baseline > $O/chunk_E.json 2> $O/chunk_E.err || { tail -20 $O/chunk_E.err; exit 4; }
python3 -c "import json;d=json.load(open('$O/chunk_E.json'));print('E', d['value'], d['kernel_us'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/chunk_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-timing > $O/chunk_prof.log 2>&1 || { tail -20 $O/chunk_prof.log; exit 6; }
find $O/chunk_prof -name "*kernel_stats.csv" | head -1 | xargs cut -c1-160 | head -8
