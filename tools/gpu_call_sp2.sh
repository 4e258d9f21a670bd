# Store policy without the asm memory clobber (in-pipeline A/B on config C),
# and the COUNT/EMIT overlap microbench with grid-strided tickets.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 200 tools/bin/overlap_ceiling > $O/overlap_ceiling.jsonl 2> $O/overlap_ceiling.err || { tail $O/overlap_ceiling.err; exit 4; }
cat $O/overlap_ceiling.jsonl
timeout -k 10 400 python3 -u tools/ab_match.py --config C --rounds 6 --steps 10 --opt nt_stores=1,3,2 > $O/ab_sp2_c.json 2> $O/ab_sp2_c.err || { tail -20 $O/ab_sp2_c.err; exit 3; }
cat $O/ab_sp2_c.json
