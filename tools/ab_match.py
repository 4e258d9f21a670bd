#!/usr/bin/env python3
"""Interleaved A/B of match-kernel options (vmqg_set_option) on one device,
one process (cdna_hip_programming.md §5.4 rule 24): the workload is loaded
once, each round runs every variant for `steps` steps; outputs are checked
equal between variants (offsets exactly, records as a per-batch checksum:
the order inside a publish may differ between variants); medians of the
per-variant step time and the COUNT / fast-EMIT kernel times are printed as
JSON.  usage: ab_match.py --config C --opt nt_stores=0,1 --opt fast_g=2,4"""
import argparse
import itertools
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--opt", action="append", default=[], help="name=v1,v2,...")
    ap.add_argument("--config", default="C", choices=["A", "C", "D", "E"])
    ap.add_argument("--e-scale", type=float, default=0.2)
    ap.add_argument("--d-scale", type=float, default=1.0)
    ap.add_argument("--n-dev", type=int, default=1_000_000)
    args = ap.parse_args()
    import torch
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    dev = torch.device("cuda", 0)
    if args.config in ("A", "C"):
        w = W.config_c(n_dev=args.n_dev) if args.config == "C" else W.config_a()
        v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes)
        w.load_into(v)
    elif args.config == "E":
        w = W.config_e(scale=args.e_scale)
        n = w.n_subs
        v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes, max_mountpoints=max(1024, len(w.mps) + 1),
                       hints={"edges": 2 * n, "paths": 2 * n, "keys": n * 5 // 4, "records": n * 5 // 4,
                              "exact": n * 5 // 4})
        w.load_into(v)
    else:
        w = W.config_d(scale=args.d_scale, n_pubs=1 << 20)
        n_live = w.notes["n_live"]
        v = RegGpuView(node=w.self_node, device=0, nodes=w.nodes,
                       hints={"edges": 4 * n_live // 5, "paths": 4 * n_live // 5, "keys": n_live,
                              "records": n_live * 11 // 10, "exact": n_live})
        w.load_into(v, n=n_live)
    pubs, words = w.publish_arrays(v)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    cap = {"A": 120, "C": 66, "D": 520, "E": 400}[args.config] * len(pubs)
    d_out = torch.empty(cap * 4, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(len(pubs) + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    names = [o.split("=")[0] for o in args.opt]
    values = [[int(x) for x in o.split("=")[1].split(",")] for o in args.opt]
    variants = list(itertools.product(*values))
    res = {str(dict(zip(names, vv))): {k: [] for k in ["step_us"] + [st + "_us" for st in v.STAGES]} for vv in variants}
    ref = None
    for rnd in range(args.rounds):
        for vv in variants:
            for n, x in zip(names, vv):
                v.set_option(n, x)
            v.match_device(d_pubs.data_ptr(), len(pubs), d_words.data_ptr(), d_out.data_ptr(), cap,
                           d_offs.data_ptr(), sp)
            torch.cuda.synchronize()
            assert v.match_status(sp) == 0, vv
            tot = int(d_offs[-1].item())
            digest = (d_offs.clone(), d_out[: 4 * tot].view(-1, 4).to(torch.int64).sum(0).cpu())
            if ref is None:
                ref = digest
            assert torch.equal(ref[0], digest[0]), ("offsets differ", vv)
            assert torch.equal(ref[1], digest[1]), ("record checksum differs", vv)
            v.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                v.match_device(d_pubs.data_ptr(), len(pubs), d_words.data_ptr(), d_out.data_ptr(), cap,
                               d_offs.data_ptr(), sp)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            stt = v.stage_times()
            v.set_timing(False)
            r = res[str(dict(zip(names, vv)))]
            r["step_us"].append(dt * 1e6)
            for st in v.STAGES:
                r[st + "_us"].append(stt[st] / 1e3)
    out = {k: {m: statistics.median(x) for m, x in d.items()} for k, d in res.items()}
    print(json.dumps({"config": args.config, "median": out, "rounds": args.rounds, "steps": args.steps}))


if __name__ == "__main__":
    main()
