"""bench.py's launcher-less `--gpus N` start (launch_ranks): N rank
processes with the environment torch.distributed.run sets, the worst exit
code returned, and a failing rank ending the others instead of leaving them
in the rendezvous.  The ranks here are stubs (a copy of bench.py whose main
only calls launch_ranks), so no GPU and no torch import is involved."""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = '''
def main():
    import argparse, json, time as _t
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--fail-rank", type=int, default=-1)
    ap.add_argument("--out", default="")
    args, _ = ap.parse_known_args()
    rc = launch_ranks(args)
    if rc is not None:
        return rc
    r = int(os.environ["RANK"])
    if args.out:
        with open("%s.%d" % (args.out, r), "w") as f:
            json.dump({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR")}, f)
    if r == args.fail_rank:
        return 3
    if args.fail_rank >= 0:
        _t.sleep(60)
    return 0
'''


def _stub_bench(tmp_path):
    src = open(os.path.join(ROOT, "bench.py")).read()
    i, j = src.index("def main():"), src.index("\nif __name__")
    p = tmp_path / "bench_stub.py"
    p.write_text(src[:i] + STUB + src[j:])
    return str(p)


def test_ranks_get_the_launcher_environment(tmp_path):
    import json
    stub = _stub_bench(tmp_path)
    out = str(tmp_path / "env")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    rc = subprocess.call([sys.executable, stub, "--gpus", "3", "--out", out], cwd=ROOT, env=env)
    assert rc == 0
    got = [json.load(open("%s.%d" % (out, r))) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"]
    assert all(g["WORLD_SIZE"] == "3" and g["MASTER_ADDR"] == "127.0.0.1" for g in got)
    assert [g["LOCAL_RANK"] for g in got] == ["0", "1", "2"]


def test_a_failing_rank_ends_the_others(tmp_path):
    stub = _stub_bench(tmp_path)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    t0 = time.time()
    rc = subprocess.call([sys.executable, stub, "--gpus", "2", "--fail-rank", "1"], cwd=ROOT, env=env, timeout=50)
    assert rc == 3                      # the failing rank's code, not the ended rank's
    assert time.time() - t0 < 30        # rank 0 (sleeping 60 s) was ended


def test_launcher_rank_count_must_match(tmp_path):
    stub = _stub_bench(tmp_path)
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert subprocess.call([sys.executable, stub, "--gpus", "4"], cwd=ROOT, env=env) == 2
