# Default bench line (config C, CPU baseline, both end-to-end modes), then a
# rocprofv3 session of the same kernels (kernel trace + PMC passes) tagged
# with the library's build id.  TAG names the profiles/ files.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench"
timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 3; }
cat gpurun_out/bench_${TAG}.json
[ -n "${NOPROF:-}" ] && exit 0
echo "== profile"
OUT=gpurun_out/prof_${TAG} TAG=${TAG} bash tools/profile_session.sh > gpurun_out/prof_${TAG}.log 2>&1 || { tail -30 gpurun_out/prof_${TAG}.log; exit 4; }
tail -5 gpurun_out/prof_${TAG}.log
