# the EMIT tail beside the fast EMIT (option tail_overlap): the whole GPU
# suite on it, then A, D (no churn) and E with it on and off on one load each
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
( while sleep 50; do date +%s >> $O/heartbeat.txt; done ) &
HB=$!
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?
kill $HB
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
for c in A D E; do
timeout -k 10 400 python -u tools/opt_sweep.py --config $c "tail_overlap=0" "tail_overlap=1" > $O/sweep_$c.jsonl 2> $O/sweep_$c.err || exit 2
done
echo done
