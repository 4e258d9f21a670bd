# the deferred-look-back fused match (K = 2) as the default: the whole GPU
# suite, then R1 and R2
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --durations=10 > $O/tests.log 2>&1
rc=$?
kill $HB
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
B="python bench.py --r-n 4096000 --no-cpu-baseline --no-e2e"
timeout -k 10 200 $B --config R1 > $O/r1.json 2>> $O/err.txt || exit 3
timeout -k 10 200 $B --config R2 > $O/r2.json 2>> $O/err.txt || exit 4
echo done
