# config C with 1, 2 and 3 matcher contexts on the GPU (consecutive steps on
# consecutive contexts / streams)
set -o pipefail
mkdir -p gpurun_out/r06j
for L in 1 2 3; do
timeout -k 10 300 python bench.py --lanes $L --no-cpu-baseline --no-e2e --steps 40 > gpurun_out/r06j/c_l$L.json 2> gpurun_out/r06j/c_l$L.err || exit $L
done
echo done
