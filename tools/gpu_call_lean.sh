# A/B: lean EMIT vs the group EMIT on configs C and D (outputs compared
# between variants inside ab_match.py), then the parity subset with lean on.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== A/B C"
timeout -k 10 300 python tools/ab_match.py --rounds 5 --steps 10 --fast-g 2 --fused 0 --lean 0,1 > gpurun_out/ab_lean_c.json 2> gpurun_out/ab_lean_c.err || { tail -20 gpurun_out/ab_lean_c.err; exit 3; }
cat gpurun_out/ab_lean_c.json
echo "== A/B D"
timeout -k 10 400 python tools/ab_match.py --config D --rounds 3 --steps 5 --fast-g 2 --fused 0 --lean 0,1 > gpurun_out/ab_lean_d.json 2> gpurun_out/ab_lean_d.err || { tail -20 gpurun_out/ab_lean_d.err; exit 4; }
cat gpurun_out/ab_lean_d.json
