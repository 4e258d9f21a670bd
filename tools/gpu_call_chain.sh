# Stream-chain ordering (no per-call event) + dispatch-recorded timing:
# every -m gpu test, config C bench line, per-call fixed cost, a kernel trace,
# and the RT / SS / AC lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
T=800 bash tools/gpu_tests.sh || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/chain_C.json 2> $O/chain_C.err || { tail -20 $O/chain_C.err; exit 2; }
python3 -c "import json;d=json.load(open('$O/chain_C.json'));print('C', d['value'], d['ms_per_step'], d.get('kernel_us'))"
timeout -k 10 240 python3 -u tools/step_overhead.py > $O/step_overhead.json 2> $O/step_overhead.err || { tail -5 $O/step_overhead.err; exit 3; }
cat $O/step_overhead.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/chain_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-timing > $O/chain_prof.log 2>&1 || { tail -20 $O/chain_prof.log; exit 4; }
for c in RT SS AC; do
  timeout -k 10 300 python3 -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > $O/chain_$c.json 2> $O/chain_$c.err || { tail -20 $O/chain_$c.err; exit 5; }
  python3 -c "import json;d=json.load(open('$O/chain_$c.json'));print('$c', d['value'], d['ms_per_step'], d.get('kernel_us'))"
done
