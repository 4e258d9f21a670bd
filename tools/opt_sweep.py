#!/usr/bin/env python3
"""Loads one workload (bench.py's configs) once and times the match under
several vmqg_set_option sets in turn (each set's options stay set for the
next: give every set the values it needs): per set, the uninstrumented ms per
step and the per-stage kernel times.  Tuning knobs only (results are
unchanged by them); one JSON line per set.

  python tools/opt_sweep.py --config E "emit_bpc=8" "emit_bpc=24" ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="E")
    ap.add_argument("--e-scale", type=float, default=1.0)
    ap.add_argument("--r-n", type=int, default=4_096_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("sets", nargs="*")
    args = ap.parse_args()
    import torch
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    if args.config == "E":
        w = W.config_e(scale=args.e_scale, n_pubs=1 << 20)
    elif args.config in ("R1", "R2"):
        w = W.CONFIGS[args.config](args.r_n)
    else:
        w = W.CONFIGS[args.config]()
    n = w.n_subs
    view = RegGpuView(node=w.self_node, device=0, nodes=w.nodes, max_mountpoints=max(1024, len(w.mps) + 1),
                      hints={"edges": 2 * n, "paths": 2 * n, "keys": n * 5 // 4, "records": n * 5 // 4, "exact": n})
    t0 = time.time()
    w.load_into(view)
    print("loaded in %.1fs" % (time.time() - t0), file=sys.stderr, flush=True)
    pubs, words = w.publish_arrays(view)
    npub = len(pubs)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    d_offs = torch.zeros(npub + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    out_cap = 16 * npub + 1024
    d_out = torch.empty(out_cap * 4, dtype=torch.int32, device=dev)
    step = lambda: view.match_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_out.data_ptr(), out_cap,
                                     d_offs.data_ptr(), sp)
    step()
    torch.cuda.synchronize()
    need = int(d_offs[-1].item())
    view.match_status(sp)
    if need > out_cap:
        out_cap = need + 1024
        d_out = torch.empty(out_cap * 4, dtype=torch.int32, device=dev)
    ref = None
    for s in ["default"] + args.sets:
        opts = [] if s == "default" else [kv.split("=") for kv in s.split(",")]
        for k, v in opts:
            view.set_option(k, int(v))
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        view.set_timing(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        stages = bench.stage_us(view)
        view.set_timing(False)
        rc = view.match_status(sp)
        offs = d_offs.cpu().numpy()
        same = ref is None or np.array_equal(offs, ref)
        ref = offs if ref is None else ref
        print(json.dumps({"set": s, "ms_per_step": el * 1e3 / args.steps, "publishes_per_s": npub * args.steps / el,
                          "kernel_us": {k: round(v, 1) for k, v in stages.items()}, "status": rc,
                          "offsets_equal": bool(same)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
