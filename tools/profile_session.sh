# rocprofv3 session for bench.py (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats; passes 2-3: one PMC counter each (never
# combined with sys/runtime traces).  Results summarised into gpurun_out/prof.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 3; }
tail -2 $OUT/stats.log
echo "== FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B --no-timing > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 4; }
echo "== WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B --no-timing > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 5; }
python3 tools/summarize_prof.py $OUT/stats $OUT/fetch $OUT/write $OUT/pmc_summary.json ${TAG:-latest}
