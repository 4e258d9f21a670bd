# Store cache policy: the microbench (store rate + what the stream does to a
# 270 MB table read next), the new parity test, then the in-pipeline A/B of
# nt_stores = 1 (nt), 0 (plain), 2 (sc1), 3 (sc1 nt) on config C.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 tools/bin/store_ceiling > $O/store_ceiling.jsonl 2> $O/store_ceiling.err || { tail $O/store_ceiling.err; exit 1; }
cat $O/store_ceiling.jsonl
timeout -k 10 200 tools/bin/overlap_ceiling > $O/overlap_ceiling.jsonl 2> $O/overlap_ceiling.err || { tail $O/overlap_ceiling.err; exit 4; }
cat $O/overlap_ceiling.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "store_policies or config_full_parity" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/sp_tests.log 2>&1 || { tail -30 $O/sp_tests.log; exit 2; }
tail -2 $O/sp_tests.log
timeout -k 10 400 python3 -u tools/ab_match.py --config C --rounds 6 --steps 10 --opt nt_stores=1,0,2,3 > $O/ab_sp_c.json 2> $O/ab_sp_c.err || { tail -20 $O/ab_sp_c.err; exit 3; }
cat $O/ab_sp_c.json
