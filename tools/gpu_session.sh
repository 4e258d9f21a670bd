set -o pipefail
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log; echo "smoke rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
echo "== gpu tests"; timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -30 gpurun_out/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
echo "== bench"; timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json; echo "bench rc=$rc"
if [ -n "$BENCH_D" ]; then
  echo "== bench D"; timeout -k 10 600 python bench.py --config D --steps 10 --warmup 2 > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err; rc=$?; tail -3 gpurun_out/bench_d.err; cat gpurun_out/bench_d.json; echo "bench D rc=$rc"
fi
exit $rc
