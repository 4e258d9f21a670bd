# rocprofv3 session for bench.py (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats; then one PMC counter group per run (never
# combined with sys/runtime traces): FETCH_SIZE, WRITE_SIZE, L2 hit/miss, LDS
# bank conflicts.  Results summarised into gpurun_out/prof.  BENCH_ARGS
# selects the workload (default: the headline config C).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-}"
export BUILD_ID=$(python3 -c "from vernemq_amd import _lib; print(_lib.build_id())")
echo "build $BUILD_ID"
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- $B > $OUT/stats.log 2>&1 || { tail -20 $OUT/stats.log; exit 3; }
tail -2 $OUT/stats.log
echo "== FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B --no-timing > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 4; }
echo "== WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B --no-timing > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 5; }
if [ -z "${LITE:-}" ]; then   # LITE=1: kernel trace + FETCH/WRITE only
echo "== L2 hit/miss"
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/l2 -o run --output-format csv -- $B --no-timing > $OUT/l2.log 2>&1 || { tail -20 $OUT/l2.log; exit 6; }
echo "== LDS bank conflicts"
timeout -k 10 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/lds -o run --output-format csv -- $B --no-timing > $OUT/lds.log 2>&1 || { tail -20 $OUT/lds.log; exit 7; }
python3 tools/summarize_prof.py $OUT/stats $OUT/fetch $OUT/write $OUT/pmc_summary.json ${TAG:-latest} $OUT/l2 $OUT/lds
else
python3 tools/summarize_prof.py $OUT/stats $OUT/fetch $OUT/write $OUT/pmc_summary.json ${TAG:-latest}
fi
