# R1 on the final build: memory-side requests and wave wait cycles of the
# fused launch (two PMC passes, nothing else traced)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
B="python3 bench.py --config R1 --r-n 4096000 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-timing"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $O/req -o run --output-format csv -- $B > $O/req.log 2>&1 || { tail -5 $O/req.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $O/sq -o run --output-format csv -- $B > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 2; }
echo done
