# Tree test, then config C bench line, per-call fixed cost, kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "tree_levels or config_d or wide_frontier" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tree_tests.log 2>&1 || { tail -40 $O/tree_tests.log; exit 1; }
tail -2 $O/tree_tests.log
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/tree_C.json 2> $O/tree_C.err || { tail -20 $O/tree_C.err; exit 2; }
python3 -c "import json;d=json.load(open('$O/tree_C.json'));print('C', d['value'], d['ms_per_step'], d.get('kernel_us'))"
timeout -k 10 240 python3 -u tools/step_overhead.py > $O/step_overhead.json 2> $O/step_overhead.err || { tail -5 $O/step_overhead.err; exit 3; }
cat $O/step_overhead.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tree_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-timing > $O/tree_prof.log 2>&1 || { tail -20 $O/tree_prof.log; exit 4; }
