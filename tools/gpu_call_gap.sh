set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/gap$m -o run --output-format csv -- python3 tools/gap_probe.py $m > gpurun_out/gap$m.log 2>&1 || { tail gpurun_out/gap$m.log; exit 1; }
  echo "== mode $m"; python3 tools/gap_report.py gpurun_out/gap$m/run_kernel_trace.csv 14
done
