# Config E at full size (50M subscriptions, 1,000 mountpoints, 12 levels) on
# one GPU: load, match, oracle sample, CPU baseline.  Progress goes to the
# .err file every ~20 s (the box kills a silent command after 180 s).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u bench.py --config E --steps 10 --warmup 2 > gpurun_out/bench_E_${TAG}.json 2> gpurun_out/bench_E_${TAG}.err || { tail -30 gpurun_out/bench_E_${TAG}.err; exit 5; }
cat gpurun_out/bench_E_${TAG}.json
tail -8 gpurun_out/bench_E_${TAG}.err
