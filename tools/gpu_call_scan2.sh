# A/B: offsets scan as one look-back launch vs reduce + scan (outputs compared
# between variants inside ab_match.py), configs C and D.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== A/B C"
timeout -k 10 300 python tools/ab_match.py --rounds 5 --steps 10 --fast-g 2 --fused 0 --scan2 0,1 > gpurun_out/ab_scan2_c.json 2> gpurun_out/ab_scan2_c.err || { tail -20 gpurun_out/ab_scan2_c.err; exit 3; }
cat gpurun_out/ab_scan2_c.json
echo "== A/B D"
timeout -k 10 400 python tools/ab_match.py --config D --rounds 3 --steps 5 --fast-g 2 --fused 0 --scan2 0,1 > gpurun_out/ab_scan2_d.json 2> gpurun_out/ab_scan2_d.err || { tail -20 gpurun_out/ab_scan2_d.err; exit 4; }
cat gpurun_out/ab_scan2_d.json
