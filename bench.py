#!/usr/bin/env python3
"""Headline benchmark: topic matches/sec (publishes/sec) at 1M subs — SURVEY.md
§8(d) config C — on 1..N MI355X, with the HIP path's roofline and the CPU
oracle (C++ restatement of vmq_reg_trie) timed beside it.

One step = one batch of 2^20 publishes (devices/{d}/telemetry/{m}) fully
matched on each GPU: count pass, offset scan, emit pass writing every
matched 16-B FoldFun record — inputs resident in HBM, outputs left in HBM.

N > 1 (launched by torch.distributed.run): the trie is built once on rank 0
and replicated by an RCCL broadcast of the device image; each rank matches
its own publish batch (weak scaling, no collective on the data path); the
per-rank emission counts are all-gathered.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def stage_us(view):
    """Average µs per launch of the five kernels of a match call (HIP events
    recorded by each dispatch): COUNT fast tier, COUNT wave tier, scan, EMIT
    fast tier, EMIT wave tier."""
    t = view.stage_times()
    out = {k: t[k] / 1e3 for k in view.STAGES}
    out["per_call"] = sum(out[k] for k in view.STAGES)
    out["launches"] = t["launches"]
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc_traffic(kernel: str, summary: str = "pmc_latest.json"):
    """HBM bytes per launch of the kernel whose name contains `kernel`
    (e.g. "k_match_fast<1" = EMIT) from a committed rocprofv3 PMC summary
    (profiles/pmc_latest.json for config C, written by
    tools/summarize_prof.py), or None.  Read bytes are 2 x FETCH_SIZE (gfx950
    correction), writes WRITE_SIZE.  The summary must have been taken on the
    library loaded now (same vmqg_build_id): a profile of other kernels is
    not evidence for these, so a mismatch reports None."""
    from vernemq_amd import _lib
    p = os.path.join(ROOT, "profiles", summary)
    try:
        doc = json.load(open(p))
        d = doc["kernels"]
    except (OSError, KeyError, ValueError):
        return None
    if doc.get("build_id") != _lib.build_id():
        log("PMC summary %s is of build %s, loaded library is %s: traffic not reported"
            % (summary, doc.get("build_id"), _lib.build_id()))
        return None
    cands = [v for k, v in d.items() if kernel in k and "hbm_bytes_per_launch" in v]
    if not cands:
        return None
    return max(cands, key=lambda v: v.get("total_ns", 0))["hbm_bytes_per_launch"]


def load_pmc_traffic_any(kernels, summary: str):
    """(name, HBM bytes per launch) of whichever of `kernels` (name
    fragments) ran longest in the PMC summary — COUNT is k_count_exact on
    trie-less tables (R1, R2), k_match_fast<0 otherwise; EMIT likewise
    k_emit_exact or k_match_fast<1 — or (None, None)."""
    best = (None, None, -1.0)
    p = os.path.join(ROOT, "profiles", summary)
    try:
        d = json.load(open(p))["kernels"]
    except (OSError, KeyError, ValueError):
        return None, None
    for kern in kernels:
        ns = max([v.get("total_ns", 0) for k, v in d.items() if kern in k] or [-1.0])
        if ns > best[2]:
            best = (kern, load_pmc_traffic(kern, summary), ns)
    return best[0], best[1]


def apply_opts(view, args):
    """--vmqg-opt NAME=VALUE knobs (vmqg_set_option: tuning only)."""
    for kv in args.vmqg_opt:
        k, v = kv.split("=", 1)
        view.set_option(k, int(v))


def launch_ranks(args):
    """`--gpus N` without a launcher: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set
    as torch.distributed.run sets them) and return the worst exit code.  The
    parent never touches the GPU (no HIP call before or after the children
    start: it only waits for them).  Under a launcher (WORLD_SIZE set) the
    launcher's rank count must equal --gpus.  Returns None when this process
    is a rank itself."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != args.gpus:
            log("--gpus %d but WORLD_SIZE=%s: the rank count must equal --gpus" % (args.gpus, world_env))
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # a rank that fails ends the others (they would wait for it in the
    # rendezvous or a collective until a watchdog fired)
    import time as _time
    rcs = [None] * len(procs)
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        _time.sleep(0.2)
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        log("rank exit codes %s" % rcs)
    # the failing rank's code, not that of a rank this parent ended
    return next((rc for rc in bad if rc > 0), 1) if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="publishes per step per GPU")
    ap.add_argument("--n-dev", type=int, default=1_000_000, help="devices/{d}/telemetry/# subscribers")
    ap.add_argument("--cpu-sample", type=int, default=100_000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline: seconds per thread count")
    ap.add_argument("--cpu-threads", type=int, default=16, help="CPU baseline: the box's host share")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="no per-launch HIP events (profiling runs)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive end-to-end figure")
    ap.add_argument("--config", default="C", choices=["A", "B", "C", "D", "E", "R1", "R2", "RT", "AC", "SS"],
                    help="C: headline (1M subs); D: 10M subs with $share groups under 1%%/s churn; "
                         "A, B, E, R1, R2: the other SURVEY §8d shapes (secondary lines); "
                         "RT: retained-message match_fold (§8f rank 3); AC: vmq_acl checks (§8f rank 4); "
                         "SS: $share dispatch on config D's match output (§8f rank 4)")
    ap.add_argument("--ac-requests", type=int, default=1 << 20, help="AC: ACL checks per step")
    ap.add_argument("--rt-devices", type=int, default=62_500, help="RT: devices x 16 retained topics")
    ap.add_argument("--rt-filters", type=int, default=1 << 18, help="RT: subscription filters per step")
    ap.add_argument("--rt-heavy", type=int, default=16, help="RT: devices/+/telemetry/{m} filters per step")
    ap.add_argument("--e-scale", type=float, default=1.0, help="config E scale (1.0 = 50M subs)")
    ap.add_argument("--fast-g", type=int, default=None,
                    help="vmqg option fast_g for the secondary configs (A/B only; default: the library's own, 1)")
    ap.add_argument("--r-n", type=int, default=1_000_000, help="R1 / R2: N (the reference suite goes to 4,096,000)")
    ap.add_argument("--exact-hint-mult", type=float, default=1.0,
                    help="A / B / R1 / R2: exact-table size hint as a multiple of the subscriptions (A/B of its load)")
    ap.add_argument("--d-scale", type=float, default=1.0)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--force-device", type=int, default=-1, help="rehearsal: every rank on this device")
    ap.add_argument("--lanes", type=int, default=1,
                    help="config C: matcher contexts on the GPU (primary + replicas), consecutive steps on "
                         "consecutive contexts and streams")
    ap.add_argument("--churn-batch", type=int, default=10_000)
    ap.add_argument("--churn-rate-batches", type=float, default=10.0, help="delta batches per second (1%%/s at 10M)")
    ap.add_argument("--vmqg-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="vmqg_set_option on every matcher context (A/B runs; results unchanged)")
    args = ap.parse_args()
    rc = launch_ranks(args)
    if rc is not None:
        return rc
    if args.config == "D":
        return bench_d(args)
    if args.config == "RT":
        return bench_retain(args)
    if args.config == "AC":
        return bench_acl(args)
    if args.config == "SS":
        return bench_shared(args)
    if args.config != "C":
        return bench_other(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.force_device >= 0:
        local = args.force_device
    import torch
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)   # RCCL on ROCm
        else:
            dist.init_process_group(args.dist_backend)

    from vernemq_amd import _lib
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView

    t0 = time.time()
    w = W.config_c(n_dev=args.n_dev, n_pubs=args.batch, seed=0xC + rank)   # same subs, per-rank publishes
    log("rank %d: workload generated in %.1fs (%d subs, %d publishes)" % (rank, time.time() - t0, w.n_subs, w.n_pubs))

    load_s = 0.0
    if rank == 0:
        t0 = time.time()
        view = RegGpuView(node=w.self_node, device=local, nodes=w.nodes,
                          hints={"edges": 3 * args.n_dev + 1024, "paths": 3 * args.n_dev + 1024,
                                 "keys": args.n_dev + 1024, "records": args.n_dev + 1024,
                                 "exact": args.n_dev + 1024})   # the filters' own local keys (fold/4 :62)
        w.load_into(view)
        load_s = time.time() - t0
        pwid = view.intern_words(w.pub_words, create=False).astype(np.int64)
        log("rank 0: initialize_trie of %d subs + device upload in %.1fs, stats %s" % (w.n_subs, load_s, view.stats_raw()))
    if world > 1:
        # replicate the trie: RCCL broadcast of the device image + layout
        # (vernemq_amd.dist.ImageSync), then of rank 0's publish word map
        from vernemq_amd import dist as vd
        if rank != 0:
            view = RegGpuView(node=w.self_node, device=local, replica=True)
        sync = vd.ImageSync(dist, view, dev)
        nbytes = sync.full()
        pw_t = torch.zeros(len(w.pub_words), dtype=torch.int64, device=dev)
        if rank == 0:
            pw_t.copy_(torch.from_numpy(pwid))
        dist.broadcast(pw_t, 0)
        pwid = pw_t.cpu().numpy()
        log("rank %d: trie image %.1f MB replicated" % (rank, nbytes / 1e6))
    apply_opts(view, args)

    pubs, words = w.publish_arrays_ids(pwid, np.array([0], dtype=np.uint32))
    npub = len(pubs)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    out_cap = (w.notes["n_wild"] + 1) * npub
    d_out = torch.empty(out_cap * 4, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(npub + 1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()
    sp = stream.cuda_stream

    def step():
        view.match_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_out.data_ptr(), out_cap,
                          d_offs.data_ptr(), sp)

    # --lanes L: L contexts on this GPU (the primary and L - 1 replicas
    # loaded from its arena, as the drop-in's view holds them), each with
    # its own stream and output buffers; consecutive steps go to
    # consecutive lanes, so one batch's COUNT can run beside another's EMIT
    lanes = [(view, stream, d_out, d_offs)]
    for _ in range(1, args.lanes):
        rv = RegGpuView(node=w.self_node, device=local, replica=True)
        ap, _, lay = view.arena()
        rv.replica_load(lay, ap, sp)
        apply_opts(rv, args)
        lanes.append((rv, torch.cuda.Stream(device=dev), torch.empty_like(d_out), torch.zeros_like(d_offs)))
    torch.cuda.synchronize()
    seq = [0]

    def step_lanes():
        v, s, o, f = lanes[seq[0] % len(lanes)]
        seq[0] += 1
        v.match_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), o.data_ptr(), out_cap, f.data_ptr(), s.cuda_stream)

    for _ in range(args.warmup):
        step()
    for _ in range(len(lanes) * max(1, args.warmup)):
        step_lanes()
    torch.cuda.synchronize()
    for v, s, _, _ in lanes:
        rc = v.match_status(s.cuda_stream)
        if rc != 0:
            raise RuntimeError("match status %d after warmup" % rc)
    # size-independent parity check of the step's output (every publish: 64
    # wildcard subscribers + its own device subscriber when d < n_dev)
    d_idx = w.pw[1::4] - 18
    want = np.where(d_idx < args.n_dev, w.notes["n_wild"] + 1, w.notes["n_wild"])
    verified = all(bool(np.array_equal(np.diff(f.cpu().numpy()), want)) for _, _, _, f in lanes)
    if not verified:
        raise RuntimeError("per-publish emission counts differ from config C's known answer")

    # `value`: the K steps with no instrumentation at all (no per-launch HIP
    # events, no per-step events), bracketed by barrier + synchronize
    view.set_timing(False)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_lanes()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
    for v, s, _, _ in lanes:
        rc = v.match_status(s.cuda_stream)
        if rc != 0:
            raise RuntimeError("match status %d in timed region" % rc)
    # a second, instrumented pass (never `value`): the per-step median SURVEY
    # §8(d) asks for, from events recorded on the launch stream between steps,
    # then the per-launch kernel times (HIP event pairs around every launch)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    evs[0].record(stream)
    for k in range(args.steps):
        step()
        evs[k + 1].record(stream)
    torch.cuda.synchronize()
    step_ms = sorted(evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps))
    median_ms = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else 0.5 * (step_ms[len(step_ms) // 2 - 1] + step_ms[len(step_ms) // 2])
    count_ns, emit_ns, nlaunch, stages = 0.0, 0.0, 0, None
    if not args.no_timing:
        view.set_timing(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        count_ns, emit_ns, nlaunch = view.kernel_times()
        stages = stage_us(view)
        view.set_timing(False)
    if view.match_status(sp) != 0:
        raise RuntimeError("match status in the instrumented pass")
    served = view.stats_raw()
    emissions = int(d_offs[-1].item())

    # SURVEY §8(d) end-to-end figure (never `value`): publishes from pinned
    # host memory, match, offsets + every record back to pinned host memory,
    # on the same stream; rank 0 at N = 1 only
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        h_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).pin_memory()
        h_words = torch.from_numpy(words.astype(np.int32)).pin_memory()
        h_offs = torch.empty(npub + 1, dtype=torch.int64).pin_memory()
        h_out = torch.empty(emissions * 4, dtype=torch.int32).pin_memory()
        cur = torch.cuda.current_stream()

        def e2e_step():
            d_pubs.copy_(h_pubs, non_blocking=True)
            d_words.copy_(h_words, non_blocking=True)
            step()
            h_offs.copy_(d_offs, non_blocking=True)
            h_out.copy_(d_out[: emissions * 4], non_blocking=True)

        e2e_step()
        cur.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            e2e_step()
        cur.synchronize()
        el_e2e = (time.perf_counter() - t0) / reps
        if view.match_status(sp) != 0 or int(h_offs[-1]) != emissions:
            raise RuntimeError("end-to-end pass differs from the device-resident one")
        pcie = h_pubs.numel() * 4 + h_words.numel() * 4 + h_offs.numel() * 8 + emissions * 16
        e2e = {"publishes_per_s": npub / el_e2e, "ms_per_batch": el_e2e * 1e3, "pcie_bytes_per_batch": pcie,
               "pcie_GBps": pcie / el_e2e / 1e9,
               "note": "H2D publishes + words, match, D2H offsets + all %d records (pinned host buffers), "
                       "same stream; bounded by PCIe, not by the kernels" % emissions}
        log("end-to-end: %.3g publishes/s (%.2f ms per batch, %.1f GB/s over PCIe)"
            % (e2e["publishes_per_s"], e2e["ms_per_batch"], e2e["pcie_GBps"]))
        del h_out
        # range mode (vmqg_match_ranges_device): one 8-B {record off, count}
        # per non-empty key + {node, 0} per remote node come back instead of
        # the records; the host walks them over its own record table
        # (vmqg_records), as the NIF does before calling FoldFun
        rng_cap = 4 * npub
        d_rng = torch.empty(rng_cap * 2, dtype=torch.int32, device=dev)
        d_roffs = torch.zeros(npub + 1, dtype=torch.int64, device=dev)
        view.match_ranges_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_rng.data_ptr(), rng_cap,
                                 d_roffs.data_ptr(), sp)
        if view.match_status(sp) != 0:
            raise RuntimeError("range-mode match status")
        n_rng = int(d_roffs[-1].item())
        h_roffs = torch.empty(npub + 1, dtype=torch.int64).pin_memory()
        h_rng = torch.empty(n_rng * 2, dtype=torch.int32).pin_memory()

        def e2e_ranges():
            d_pubs.copy_(h_pubs, non_blocking=True)
            d_words.copy_(h_words, non_blocking=True)
            view.match_ranges_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_rng.data_ptr(), rng_cap,
                                     d_roffs.data_ptr(), sp)
            h_roffs.copy_(d_roffs, non_blocking=True)
            h_rng.copy_(d_rng[: n_rng * 2], non_blocking=True)

        e2e_ranges()
        cur.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            e2e_ranges()
        cur.synchronize()
        el_r = (time.perf_counter() - t0) / reps
        if view.match_status(sp) != 0 or int(h_roffs[-1]) != n_rng:
            raise RuntimeError("range-mode end-to-end pass failed")
        # the ranges expand to exactly the records of the device-resident pass
        rng_np = h_rng.numpy().view(np.uint32).reshape(-1, 2)
        want_cnt = np.diff(d_offs.cpu().numpy())
        got_cnt = np.zeros(npub, dtype=np.int64)
        per = np.where(rng_np[:, 1] > 0, rng_np[:, 1], 1).astype(np.int64)
        np.add.at(got_cnt, np.repeat(np.arange(npub), np.diff(h_roffs.numpy())), per)
        if not np.array_equal(got_cnt, want_cnt):
            raise RuntimeError("range-mode entries do not expand to the record-mode counts")
        pcie_r = h_pubs.numel() * 4 + h_words.numel() * 4 + h_roffs.numel() * 8 + n_rng * 8
        e2e["ranges"] = {"publishes_per_s": npub / el_r, "ms_per_batch": el_r * 1e3, "pcie_bytes_per_batch": pcie_r,
                         "pcie_GBps": pcie_r / el_r / 1e9, "entries_per_batch": n_rng,
                         "note": "vmqg_match_ranges_device: H2D publishes + words, match, D2H offsets + %d "
                                 "{record off, count} / {node, 0} entries (pinned host buffers, same stream); "
                                 "records are read on the host from vmqg_records" % n_rng}
        log("end-to-end (ranges): %.3g publishes/s (%.2f ms per batch, %d entries)"
            % (npub / el_r, el_r * 1e3, n_rng))

    # max over ranks of the timed region; all-gather the per-GPU match counts
    t_max = elapsed
    total_emit = emissions * args.steps
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        allc = vd.gather_counts(dist, [npub * args.steps, emissions * args.steps], dev)   # per-GPU counts
        total_emit = int(allc[:, 1].sum())
    total_pubs = npub * args.steps * world
    value = total_pubs / t_max

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import feed   # the CPU restatement: baseline only, never the measured path
        t0 = time.time()
        orc = feed.load(w)
        log("cpu baseline: oracle loaded %d subs in %.1fs" % (w.n_subs, time.time() - t0))
        S = min(args.cpu_sample, npub)
        buf = feed.publish_bytes(w, 0, S)
        # 1 thread and the box's host share (16 threads; the
        # tables shared read-only, publishes partitioned — ETS read_concurrency)
        rates = {}
        for th in (1, args.cpu_threads):
            ns1, _ = orc.fold_timed(buf, 1, th)
            reps = max(1, int(math.ceil(args.cpu_seconds * 1e9 / max(ns1, 1))))
            ns, em = orc.fold_timed(buf, reps, th)
            rates[th] = (S * reps / (ns / 1e9), reps, ns / 1e9)
            log("cpu baseline: %d thread(s) %.0f publishes/s" % (th, rates[th][0]))
        th = args.cpu_threads
        cpu = {"value": rates[th][0], "unit": "publishes/s", "cores": th, "kind": "port",
               "single_thread_value": rates[1][0],
               "sample": "first %d publishes of the config-C step batch x %d reps (%.1fs) on %d threads (publishes "
                         "partitioned, tables shared read-only; 1 thread: %.3g publishes/s), "
                         "oracle/vmq_trie_oracle.cpp (C++ restatement of vmq_reg_trie fold/4 over "
                         "hash-map 'ETS' tables, not BEAM); host %s"
                         % (S, rates[th][1], rates[th][2], th, rates[1][0], cpu_model())}

    if rank == 0:
        # roofline of the dominant kernel (EMIT): its compulsory HBM bytes per
        # launch (records written + key cache / offsets read + each distinct
        # record read once, W.algorithmic_bytes_c "emit_compulsory") over its
        # average launch time from HIP events on the launch stream.  SURVEY
        # §8(d)'s B_p (16-B lookups + 32 B per emission) is reported as
        # `survey_model`: it charges an HBM read for every emission of the
        # L2-resident fan-out list, so it can exceed what the chip moves.
        alg = {"count": W.algorithmic_bytes_c(w, part="lookup"), "emit": W.algorithmic_bytes_c(w, part="emit"),
               "count_tx": W.algorithmic_bytes_c(w, part="lookup_tx"),
               "all": W.algorithmic_bytes_c(w), "emit_compulsory": W.algorithmic_bytes_c(w, part="emit_compulsory")}
        kern = "k_match_fast<1"
        achieved = alg["emit_compulsory"] / emit_ns if emit_ns > 0 else None   # bytes/ns == GB/s
        traffic = load_pmc_traffic(kern)
        pipe_ns = t_max * 1e9 / args.steps
        res = {
            "metric": "topic matches/sec (publishes/sec) at 1M subs, 1/2/4/8 MI355X vs CPU trie",
            "value": value,
            "unit": "publishes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max * 1e3 / args.steps,
            "median_ms_per_step": median_ms,
            "median_publishes_per_s": npub * world / (median_ms / 1e3),
            "timing_note": "value: K uninstrumented steps between barrier + synchronize; median: a second pass "
                           "with one event per step boundary; kernel_us: a third pass with HIP event pairs "
                           "around every launch",
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: SURVEY.md §8(d) config C generator (splitmix64 seed 0xC + rank)",
            "config": {"workload": "C: %d subs (devices/{d}/telemetry/# x %d + devices/+/telemetry/# x %d), "
                                   "%d publishes/step/GPU devices/{d}/telemetry/{m}, d < %d"
                                   % (w.n_subs, args.n_dev, w.notes["n_wild"], npub, int(args.n_dev * 1.25)),
                       "subs": w.n_subs, "publishes_per_step_per_gpu": npub,
                       "parallelism": "trie replicated (RCCL broadcast), publishes sharded x%d" % world,
                       "contexts_per_gpu": len(lanes)},
            "pairs_per_s": total_emit / t_max,
            "emissions_per_step_per_gpu": emissions,
            "verified_counts": verified,
            "kernel_us": stages,
            "served": {"deferred": served["deferred_tier1"], "retried": served["retried"], "many_key": served["many_key"],
                       "wave_entries": served["wave_entries"], "wide_entries": served["wide_entries"],
                       "dedup": served["dedup"], "dedup_walked": served["dedup_walked"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": (achieved / PEAK_HBM_GBS) if achieved else None, "traffic": traffic,
                         "frac_physical": traffic / emit_ns / PEAK_HBM_GBS if traffic and emit_ns > 0 else None,
                         "kernel": "k_match_fast<1,0,2,true,64> (EMIT)",
                         "algorithmic_bytes_per_launch": alg["emit_compulsory"],
                         "bytes_model": "16 B written per emission + 40 B read per publish + 16 B per distinct "
                                        "record (workloads.algorithmic_bytes_c emit_compulsory)"},
            "count_kernel": {"kernel": "k_match_fast<0,0,1,true,64> (COUNT)", "us": count_ns / 1e3 if count_ns else None,
                             "lookup_bytes_model": alg["count"],
                             "achieved": alg["count"] / count_ns if count_ns else None,
                             "lookup_tx_bytes": alg["count_tx"],
                             "achieved_tx": alg["count_tx"] / count_ns if count_ns else None,
                             "tx_note": "SURVEY 8(d) transaction-granular figure: each of the reference's logical "
                                        "lookups charged a whole 64-B line; above the HBM peak because the walk "
                                        "resolves most of them without a random line (edge flags, '#' alias "
                                        "records, the L2-resident devices/+ branch): 3 random lines per hit "
                                        "publish, 52 G random probes/s measured ceiling (DESIGN.md)"},
            "survey_model": {"bytes_per_step": alg["all"], "achieved_per_step": alg["all"] / pipe_ns,
                             "emit_achieved": alg["emit"] / emit_ns if emit_ns else None,
                             "note": "SURVEY 8(d) B_p = 8(L+1) + 16 S_p + 32 R_p; charges an HBM read per emission "
                                     "of the cache-resident fan-out list, so it can exceed the HBM peak"},
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "load_s": load_s,
            "build_id": _lib.build_id(),
        }
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


def bench_other(args):
    """Secondary lines: configs A, B, E and the reference's
    bench shapes R1 / R2 (vmq_reg_trie_bench_SUITE.erl:97-214) on one GPU.
    Each line carries the dominant kernel's roofline and the CPU
    restatement timed on a bounded sample, whose publishes are also checked
    against the oracle publish for publish.  Config E at full size (50M
    subscriptions over 1,000 mountpoints) cannot be held by the oracle:
    its sample is the batch's first publishes in mountpoints of <= 2M
    subscriptions, and the oracle holds exactly those mountpoints'
    subscriptions (a publish only walks its own mountpoint's trie, so the
    check is exact at full scale)."""
    import torch
    from oracle import oracle as O
    from vernemq_amd import _lib
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t0 = time.time()
    if args.config == "E":
        log("config E: generating %.0fM subscriptions" % (50 * args.e_scale))
        w = W.config_e(scale=args.e_scale, n_pubs=args.batch)
    elif args.config in ("R1", "R2"):
        w = W.CONFIGS[args.config](args.r_n)
    else:
        w = W.CONFIGS[args.config]()
    gen_s = time.time() - t0
    n = w.n_subs
    # the exact table holds every topic with a local key or remote entries (at
    # most one per subscription): sized for n, it is planned at load <= 0.25
    hints = {"edges": 2 * n, "paths": 2 * n, "keys": n * 5 // 4, "records": n * 5 // 4,
             "exact": int(n * args.exact_hint_mult)}
    view = RegGpuView(node=w.self_node, device=0, nodes=w.nodes, max_mountpoints=max(1024, len(w.mps) + 1),
                      hints=hints)
    t0 = time.time()
    last = [t0]

    def progress(done, total):
        if time.time() - last[0] > 20:
            last[0] = time.time()
            log("config %s: %d / %d subscriptions loaded (%.0fs)" % (args.config, done, total, time.time() - t0))

    apply_opts(view, args)   # layout knobs ("exact_one") take effect on the load
    w.load_into(view, progress=progress)
    load_s = time.time() - t0
    fast_g = args.fast_g
    if fast_g:
        view.set_option("fast_g", fast_g)
    apply_opts(view, args)
    st = view.stats_raw()
    log("config %s: %d subs generated in %.1fs, loaded in %.1fs (host engine %.1fs), %s"
        % (args.config, n, gen_s, load_s, st["apply_host_ns"] / 1e9, st))
    pubs, words = w.publish_arrays(view)
    npub = len(pubs)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    d_offs = torch.zeros(npub + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    out_cap = 16 * npub + 1024
    d_out = torch.empty(out_cap * 4, dtype=torch.int32, device=dev)
    view.match_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_out.data_ptr(), out_cap, d_offs.data_ptr(), sp)
    torch.cuda.synchronize()
    need = int(d_offs[-1].item())
    view.match_status(sp)
    if need > out_cap:
        out_cap = need + 1024
        d_out = torch.empty(out_cap * 4, dtype=torch.int32, device=dev)
    step = lambda: view.match_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_out.data_ptr(), out_cap,
                                     d_offs.data_ptr(), sp)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if view.match_status(sp) != 0:
        raise RuntimeError("match status after warmup")
    # value from uninstrumented steps; kernel times from a second pass
    view.set_timing(False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if view.match_status(sp) != 0:
        raise RuntimeError("match status in timed region")
    count_ns, emit_ns, stages = 0.0, 0.0, None
    if not args.no_timing:
        view.set_timing(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        count_ns, emit_ns, _ = view.kernel_times()
        stages = stage_us(view)
        view.set_timing(False)
        if view.match_status(sp) != 0:
            raise RuntimeError("match status in the instrumented pass")
    em = int(d_offs[-1].item())
    st = view.stats_raw()
    offs_h = d_offs.cpu().numpy()

    # oracle leg: parity on a sample, lookup counts (SURVEY B_p), CPU baseline
    cpu, parity, b_p = None, None, None
    if not args.no_cpu_baseline:
        # bounded sample: <= 2,048 publishes and <= 4M emissions (R2's one
        # publish emits every subscriber)
        CS = int(max(1, min(2048, npub, np.searchsorted(offs_h, 4_000_000, side="right") - 1)))
        if w.clients is None:
            per_mp = np.bincount(w.client_mp, minlength=len(w.mps))
            small = per_mp <= 2_000_000
            cand = np.flatnonzero(small[w.pub_mp])[:CS]
            mps = np.unique(w.pub_mp[cand])
            subs_idx = np.flatnonzero(np.isin(w.client_mp[w.sub_client], mps))
            sample_note = ("%d publishes of the batch in %d mountpoints of <= 2M subscriptions; the oracle holds "
                           "those mountpoints' %d subscriptions" % (len(cand), len(mps), len(subs_idx)))
        else:
            cand = np.arange(CS)
            subs_idx = None
            sample_note = "first %d publishes of the batch against all %d subscriptions" % (CS, n)
        from oracle import feed   # the CPU restatement: checker, lookup counts and baseline only
        t0 = time.time()
        orc = O.TrieOracle(w.self_node)
        B = 1 << 18
        idx_all = np.arange(n) if subs_idx is None else subs_idx
        for lo in range(0, len(idx_all), B):
            orc.apply_raw(feed.init_bytes(w, idx=idx_all[lo:lo + B]))
            log("oracle: %d / %d subscriptions loaded (%.0fs)" % (min(len(idx_all), lo + B), len(idx_all),
                                                                 time.time() - t0))
        want, counts = orc.fold_batch([(w.mps[w.pub_mp[i]], b"pub", w.pub_topic(i)) for i in cand], with_counts=True)
        recs = d_out[: int(offs_h[-1]) * 4].cpu().numpy().view(np.uint32).reshape(-1, 4)
        infos = view.subinfos.terms
        bad = 0
        for j, i in enumerate(cand):
            got = []
            for r in recs[int(offs_h[i]):int(offs_h[i + 1])]:
                kind, node = int(r[0]) >> 24, int(r[0]) & 0xFFFFFF
                if kind == _lib.EMIT_LOCAL:
                    sid = w.client_term(int(r[2])) if w.clients is None else view.subscribers.terms[r[2]]
                    got.append(("A", sid, O.subinfo_repr(infos[r[3]])))
                elif kind == _lib.EMIT_GROUP:
                    sid = w.client_term(int(r[2])) if w.clients is None else view.subscribers.terms[r[2]]
                    got.append(("B", view.nodes.terms[node], view.word_text(int(r[1])), sid,
                                O.subinfo_repr(infos[r[3]])))
                else:
                    got.append(("C", view.nodes.terms[node]))
            bad += sorted(got) != sorted(want[j])
        parity = {"publishes": len(cand), "differ": bad, "sample": sample_note}
        if bad:
            raise RuntimeError("config %s: %d of %d sampled publishes differ from the oracle" % (args.config, bad, len(cand)))
        b_p = {"lookup": float(np.mean([8 * (c[2] + 1) + 16 * c[0] for c in counts])),
               "emit": float(np.mean([32 * c[1] for c in counts]))}
        buf = feed.publish_bytes(w, 0, 0, idx=cand)
        rates = {}
        for th in (1, args.cpu_threads):
            ns1, _ = orc.fold_timed(buf, 1, th)
            reps = max(1, int(math.ceil(args.cpu_seconds * 1e9 / max(ns1, 1))))
            ns, _ = orc.fold_timed(buf, reps, th)
            rates[th] = (len(cand) * reps / (ns / 1e9), reps, ns / 1e9)
        cpu = {"value": rates[args.cpu_threads][0], "unit": "publishes/s", "cores": args.cpu_threads, "kind": "port",
               "single_thread_value": rates[1][0],
               "sample": "%s; x %d reps (%.1fs) on %d threads (1 thread: %.3g publishes/s); oracle/vmq_trie_oracle.cpp "
                         "(C++ restatement of vmq_reg_trie fold/4; not BEAM); host %s"
                         % (sample_note, rates[args.cpu_threads][1], rates[args.cpu_threads][2], args.cpu_threads,
                            rates[1][0], cpu_model())}
        del orc

    # roofline of the dominant kernel: COUNT with SURVEY §8(d)'s lookup bytes
    # 8(L+1) + 16 S_p (S_p from the oracle's counters on the sample), or EMIT
    # with its compulsory bytes: 16 B written per emission, the 8-B offset and
    # the 32-B key cache per publish (the records it copies are read from
    # lists that many publishes share, so they are not priced per emission;
    # SURVEY's 32 B per emission is reported beside as survey_model_*).  When
    # the EMIT tail outweighs the fast EMIT (R2: one publish of 4,096,000
    # records, copied by every wave of the tail), the two EMIT launches are
    # priced together.  frac_physical = the PMC HBM bytes of the same build
    # (profiles/pmc_<config>.json) over the same time.
    roof = None
    tail_ns = stages["emit_wave"] * 1e3 if stages else 0.0
    if count_ns or emit_ns:
        pmc = "pmc_%s.json" % args.config.lower()
        survey = None
        fused = bool(stages) and stages["scan"] == 0 and stages["emit"] == 0 and count_ns > 0
        if fused and count_ns >= tail_ns:
            # trie-less tables: COUNT, scan and EMIT are one launch
            # (k_match_exact_fused), priced with all three's compulsory bytes
            alg = (b_p["lookup"] + 8) * npub + 16 * em if b_p else None
            kn, traffic = load_pmc_traffic_any(["k_match_exact_fused"], pmc)
            kern, ns = "k_match_exact_fused (COUNT + scan + EMIT)", count_ns
            model = ("8(L+1) + 16 S_p per publish (lookup, S_p averaged over the oracle sample) + 8-B offset per "
                     "publish + 16 B written per emission")
        elif count_ns >= emit_ns + tail_ns:
            alg = b_p["lookup"] * npub if b_p else None
            kn, traffic = load_pmc_traffic_any(["k_match_fast<0", "k_count_exact"], pmc)
            kern, ns, model = "%s,...> (COUNT)" % (kn or "k_match_fast<0"), count_ns, \
                "8(L+1) + 16 S_p per publish, S_p averaged over the oracle sample"
        elif emit_ns >= tail_ns:
            alg, survey = 16 * em + 40 * npub, 32 * em
            kn, traffic = load_pmc_traffic_any(["k_match_fast<1", "k_emit_exact"], pmc)
            kern, ns = "%s,...> (EMIT)" % (kn or "k_match_fast<1"), emit_ns
            model = "16 B written per emission + 8-B offset and 32-B key cache per publish"
        elif fused:   # R2: the fused match hands its one huge publish to the tail, which writes it
            alg, survey = 16 * em + 40 * npub, 32 * em
            kern, ns = "EMIT tail (k_match_wave<1>, after k_match_exact_fused)", tail_ns
            model = "16 B written per emission + 8-B offset and 32-B key cache per publish"
            traffic = load_pmc_traffic("k_match_wave<1", pmc)
        else:
            alg, survey = 16 * em + 40 * npub, 32 * em
            kn, t1 = load_pmc_traffic_any(["k_match_fast<1", "k_emit_exact"], pmc)
            kern, ns = "EMIT + EMIT tail (%s> + k_match_wave<1>, per call)" % (kn or "k_match_fast<1"), emit_ns + tail_ns
            model = "16 B written per emission + 8-B offset and 32-B key cache per publish, both EMIT launches"
            t2 = load_pmc_traffic("k_match_wave<1", pmc)
            traffic = t1 + t2 if t1 is not None and t2 is not None else None
        ach = alg / ns if alg else None
        roof = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": ach / PEAK_HBM_GBS if ach else None, "traffic": traffic,
                "frac_physical": traffic / ns / PEAK_HBM_GBS if traffic else None,
                "kernel": kern, "kernel_us": ns / 1e3, "algorithmic_bytes_per_launch": alg, "bytes_model": model,
                "survey_model_bytes": survey,
                "survey_model_frac": survey / ns / PEAK_HBM_GBS if survey else None}
    print(json.dumps({
        "metric": "publishes/sec (config %s)" % args.config, "value": npub * args.steps / el, "unit": "publishes/s",
        "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": el * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: SURVEY.md §8(d) config %s generator" % args.config,
        "config": {"workload": "%s: %d subs, %d publishes per step%s"
                               % (args.config, n, npub, ", %d mountpoints" % len(w.mps) if len(w.mps) > 1 else ""),
                   "fast_g": fast_g or "auto"},
        "pairs_per_s": em * args.steps / el, "emissions_per_step": em,
        "kernel_us": stages,
        "roofline": roof, "survey_bytes_per_publish": b_p, "oracle_sample": parity, "cpu_baseline": cpu,
        "generate_s": gen_s, "load_s": load_s, "load_host_engine_s": st["apply_host_ns"] / 1e9,
        "arena_bytes": st["device_bytes"], "trie_edges": st["trie_edges"], "paths": st["paths"],
        "rebuilds": st["rebuilds"], "deferred": [st["deferred_tier1"], st["deferred_tier2"]],
        "served": {"deferred": st["deferred_tier1"], "retried": st["retried"],
                   "many_key": st["many_key"], "wave_entries": st["wave_entries"], "wide_entries": st["wide_entries"],
                   "dedup": st["dedup"], "dedup_walked": st["dedup_walked"]},
        "build_id": _lib.build_id()}), flush=True)


def _dist_init(args):
    """RANK / LOCAL_RANK / WORLD_SIZE from torch.distributed.run; nccl = RCCL."""
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.force_device >= 0:
        local = args.force_device
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    return world, rank, local, dev, dist


def bench_d(args):
    """Config D: 10M subscriptions (8M exact, 1M '+'/'#', 1M
    $share members on 4 nodes) under 1 %/s churn: 10 delta batches per second
    of 10k ops (50/50 sub/unsub).  One step = one churn period: every rank
    queues the match batches (2^20 publishes each) that fit in 100 ms of its
    GPU time, then rank 0 applies the period's delta batch in the host
    engine (vmqg_apply_ops: never waits for the queued matches; its patches
    land after them, stream-ordered) and, at N > 1, broadcasts the patches to
    every replica over RCCL (ImageSync.delta, sizes over a host gloo group).
    At the end every rank matches one common sample batch: replica outputs
    must equal rank 0's byte for byte, and the per-publish counts the known
    answer of the live set (workloads.config_d_counts)."""
    import hashlib

    import torch
    world, rank, local, dev, dist = _dist_init(args)
    from vernemq_amd import _lib
    from vernemq_amd import dist as vd
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    t0 = time.time()
    w = W.config_d(scale=args.d_scale, n_pubs=args.batch)
    n_live = w.notes["n_live"]
    load_s = 0.0
    ch = W.Churn(w)
    if rank == 0:
        view = RegGpuView(node=w.self_node, device=local, nodes=w.nodes,
                          hints={"edges": 4 * n_live // 5, "paths": 4 * n_live // 5, "keys": n_live,
                                 "records": n_live * 11 // 10, "exact": n_live})
        ids = w.load_into(view, n=n_live)
        load_s = time.time() - t0
        log("config D: %d live subs loaded in %.1fs, %s" % (n_live, load_s, view.stats_raw()))
        pwid = view.intern_words(w.pub_words, create=False).astype(np.int64)
    else:
        view = RegGpuView(node=w.self_node, device=local, replica=True)
        pwid = np.zeros(len(w.pub_words), dtype=np.int64)
    sync = None
    if world > 1:
        sync = vd.ImageSync(dist, view, dev)
        nbytes = sync.full()
        pw_t = torch.from_numpy(pwid).to(dev)
        dist.broadcast(pw_t, 0)
        pwid = pw_t.cpu().numpy()
        log("rank %d: config D image %.1f MB replicated" % (rank, nbytes / 1e6))
    apply_opts(view, args)
    pubs, words = w.publish_arrays_ids(pwid, np.array([0], dtype=np.uint32))
    npub = len(pubs)
    pubs0 = pubs
    if rank:   # every GPU its own batch of the same distribution
        pubs = np.roll(pubs, rank * npub // world)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    d_offs = torch.zeros(npub + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    out_cap = 1024
    d_out = torch.empty(out_cap * 4, dtype=torch.int32, device=dev)

    def match():
        view.match_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_out.data_ptr(), out_cap,
                          d_offs.data_ptr(), sp)

    match()   # sizes the output (the churn keeps the total within 20 %)
    torch.cuda.synchronize()
    need = int(d_offs[-1].item())
    view.match_status(sp)
    out_cap = int(need * 1.2) + 1024
    d_out = torch.empty(out_cap * 4, dtype=torch.int32, device=dev)
    batches = [ch.batch(args.churn_batch) for _ in range(args.warmup + args.steps)]
    # the delta batches' op arrays (what the NIF builds from subscriber events)
    # are made before the timed loop: numpy gathers over the 10M-row workload
    # would otherwise evict the host engine's tables between batches
    op_arrays = [ch.ops(ids, *b) for b in batches] if rank == 0 else None
    ops_of = (lambda k: op_arrays[k]) if rank == 0 else None

    def period(k, per_period, acc):
        for _ in range(per_period):
            match()                                   # queued on the GPU
        if rank == 0:
            ops, wds = ops_of(k)
            ta = time.perf_counter()
            view.apply_op_arrays(ops, wds)            # host engine; patches queued behind the matches
            acc["apply"] += time.perf_counter() - ta
        if sync is not None:
            td = time.perf_counter()
            acc["patches"] += max(0, sync.delta())
            acc["delta"] += time.perf_counter() - td

    acc = {"apply": 0.0, "delta": 0.0, "patches": 0}
    for k in range(args.warmup):
        period(k, 1, acc)
    torch.cuda.synchronize()
    if view.match_status(sp) != 0:
        raise RuntimeError("match status after warmup")
    # GPU time of one match batch -> match batches per 100 ms churn period (rank 0 decides)
    t0 = time.perf_counter()
    for _ in range(5):
        match()
    torch.cuda.synchronize()
    t_match = (time.perf_counter() - t0) / 5
    period_s = 1.0 / args.churn_rate_batches
    pp = torch.tensor([max(1, int(period_s / t_match))], dtype=torch.int64, device=dev)
    if dist:
        dist.broadcast(pp, 0)
    per_period = int(pp.item())
    log("rank %d: match batch %.2f ms -> %d match batches per %.0f ms churn period"
        % (rank, t_match * 1e3, per_period, period_s * 1e3))
    st0 = view.stats_raw()
    view.set_timing(False)   # `value` from uninstrumented periods; kernel times from a pass after
    acc = {"apply": 0.0, "delta": 0.0, "patches": 0}
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        period(k, per_period, acc)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist:
        dist.barrier()
    rc = view.match_status(sp)
    if rc != 0:
        raise RuntimeError("match status %d" % rc)
    st1 = view.stats_raw()   # how the last timed batch was served (deferred / many-key / wave-tier entries)
    view.set_timing(True)    # the instrumented pass: per-launch times of 5 match batches
    for _ in range(5):
        match()
    torch.cuda.synchronize()
    count_ns, emit_ns, _ = view.kernel_times()
    stages = stage_us(view)
    view.set_timing(False)
    if view.match_status(sp) != 0:
        raise RuntimeError("match status (instrumented pass)")
    emitted = int(d_offs[-1].item())
    # parity: every rank matches rank 0's (unrolled) batch; replicas must
    # equal the primary byte for byte, and all the live set's known answer
    if rank:
        d_pubs.copy_(torch.from_numpy(pubs0.view(np.uint32).reshape(-1).copy()))
    match()
    torch.cuda.synchronize()
    if view.match_status(sp) != 0:
        raise RuntimeError("match status (parity pass)")
    offs_h = d_offs.cpu().numpy()
    want_counts = W.config_d_counts(w, ch.live)
    known = bool(np.array_equal(np.diff(offs_h), want_counts))
    images_equal = True
    if dist:   # every replica's device arena must equal the primary's, region by region
        regions = vd.arena_region_hashes(view, dev)
        allr = vd.gather_counts(dist, np.array(regions, dtype=np.int64), dev)
        images_equal = bool((allr == allr[0]).all())
        if not images_equal:
            log("rank %d: arena regions differing from rank 0: %s" % (rank, [
                vd.REGION_NAMES[i] for i in range(len(regions)) if (allr[:, i] != allr[0, i]).any()]))
    if not known:
        bad = np.flatnonzero(np.diff(offs_h) != want_counts)
        raise RuntimeError("rank %d: config D counts differ from the live set's known answer at %d of %d publishes "
                           "(first %s: got %s, want %s); replica images equal: %s"
                           % (rank, len(bad), npub, bad[:4].tolist(), np.diff(offs_h)[bad[:4]].tolist(),
                              want_counts[bad[:4]].tolist(), images_equal))
    if not images_equal:
        raise RuntimeError("replica arena image differs from the primary's")
    S = min(npub, 1 << 16)
    h = hashlib.sha256(offs_h[: S + 1].tobytes() + d_out[: int(offs_h[S]) * 4].cpu().numpy().tobytes()).digest()
    replicas_equal = True
    if dist:
        allh = vd.gather_counts(dist, np.frombuffer(h[:16], dtype=np.int64), dev)
        replicas_equal = bool((allh == allh[0]).all())
        if not replicas_equal:
            raise RuntimeError("replica match output differs from the primary's")
    t_max = el
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    total_pubs = npub * args.steps * per_period * world

    cpu = None
    b_p = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import feed   # the CPU restatement: baseline (and lookup counts) only
        t0 = time.time()
        orc = feed.load_prefix(w, n_live)
        log("D cpu baseline: oracle loaded %d subs in %.1fs" % (n_live, time.time() - t0))
        CS = 2048
        buf = feed.publish_bytes(w, 0, CS)
        rates = {}
        for th in (1, args.cpu_threads):
            ns1, _ = orc.fold_timed(buf, 1, th)
            reps = max(1, int(math.ceil(args.cpu_seconds * 1e9 / max(ns1, 1))))
            ns, _ = orc.fold_timed(buf, reps, th)
            rates[th] = (CS * reps / (ns / 1e9), reps, ns / 1e9)
        _, counts = orc.fold_batch([("", b"p", w.pub_topic(i)) for i in range(256)], with_counts=True)
        b_p = {"lookup": float(np.mean([8 * (c[2] + 1) + 16 * c[0] for c in counts])),
               "emit": float(np.mean([32 * c[1] for c in counts]))}
        cpu = {"value": rates[args.cpu_threads][0], "unit": "publishes/s", "cores": args.cpu_threads, "kind": "port",
               "single_thread_value": rates[1][0],
               "sample": "first %d publishes of the D batch x %d reps (%.1fs) on %d threads against the %d live "
                         "subscriptions (1 thread: %.3g publishes/s), oracle/vmq_trie_oracle.cpp (C++ restatement "
                         "of vmq_reg_trie fold/4; not BEAM); host %s"
                         % (CS, rates[args.cpu_threads][1], rates[args.cpu_threads][2], args.cpu_threads, n_live,
                            rates[1][0], cpu_model())}
        log("D cpu baseline: %.0f publishes/s (%d threads), %.0f (1 thread)"
            % (rates[args.cpu_threads][0], args.cpu_threads, rates[1][0]))

    if rank == 0:
        ops_n = st1["ops_applied"] - st0["ops_applied"]
        wait_ns = st1["apply_wait_ns"] - st0["apply_wait_ns"]
        # host work: apply_host_ns times the host stage alone (ABI 6: the
        # device commit, where GPU back-pressure waits, is timed apart)
        host_ns = st1["apply_host_ns"] - st0["apply_host_ns"]
        # Each EMIT launch is charged only the records it writes (counted on
        # the device): the fast EMIT launch writes every publish's records
        # except the wide ones' ($share groups on 4 nodes: 40 keys; alarm
        # lists: 1,000 records) and the whole-wave walks', which the EMIT
        # tail launch writes (stats wide_entries, wave_entries).  Compulsory
        # HBM bytes = 16 B written per record (the records read are the 16 MB
        # of $share member lists, the 16 MB of alarm lists and the exact
        # keys' records, cache-resident); SURVEY §8(d)'s 32 B per emission is
        # reported beside it.  The roofline line is the longer launch.
        wave_rec = int(st1["wave_entries"])
        wide_rec = int(st1["wide_entries"])
        fast_rec = emitted - wave_rec - wide_rec
        per_kernel = {
            "emit": {"kernel": "k_match_fast<1,0,2,true,64> (EMIT fast tier)", "records": fast_rec,
                     "bytes": 16 * fast_rec, "us": stages["emit"]},
            "emit_tail": {"kernel": "k_match_wave<1,0,true> (EMIT tail: wide publishes + whole-wave walks)",
                          "records": wide_rec + wave_rec, "wide_records": wide_rec, "walked_records": wave_rec,
                          "bytes": 16 * (wide_rec + wave_rec), "us": stages["emit_wave"]},
        }
        for v in per_kernel.values():
            v["GBps"] = v["bytes"] / (v["us"] * 1e3) if v["us"] else None
            v["frac"] = v["GBps"] / PEAK_HBM_GBS if v["GBps"] else None
        dom_key = max(per_kernel, key=lambda k: per_kernel[k]["us"])
        dom = per_kernel[dom_key]
        d_traffic = load_pmc_traffic("k_match_fast<1" if dom_key == "emit" else "k_match_wave<1", "pmc_d.json")
        alg_emit = dom["bytes"]
        achieved = dom["GBps"]
        step_level = {"bytes_written": 16 * emitted, "gpu_us_per_batch": stages["per_call"],
                      "GBps": 16 * emitted / (stages["per_call"] * 1e3) if stages["per_call"] else None}
        res = {
            "metric": "publishes/sec under churn (config D, 10M subs incl. $share, 1%/s deltas)",
            "value": total_pubs / t_max, "unit": "publishes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": t_max * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: SURVEY.md §8(d) config D generator (splitmix64 seed 0xD), scale %g" % args.d_scale,
            "config": {"workload": "D: %d live subs, %d-op delta batch per period (%g periods/s) + %d match "
                                   "batches of %d publishes per period per GPU"
                                   % (n_live, args.churn_batch, args.churn_rate_batches, per_period, npub),
                       "parallelism": "trie replicated, deltas broadcast as patches (RCCL), publishes sharded x%d"
                                      % world},
            "deltas_per_s": args.churn_batch * args.steps / t_max,
            "delta_apply": {"host_ops_per_s": ops_n / (host_ns / 1e9) if host_ns else None,
                            "host_ms_per_batch": host_ns / 1e6 / args.steps,
                            "enqueue_ms_per_batch": (st1["apply_upload_ns"] - st0["apply_upload_ns"] - wait_ns)
                                                    / 1e6 / args.steps,
                            "backpressure_ms_per_batch": wait_ns / 1e6 / args.steps,
                            "caller_ms_per_batch": acc["apply"] * 1e3 / args.steps,
                            "patch_bytes_per_batch": (st1["patch_bytes"] - st0["patch_bytes"]) / args.steps,
                            "full_images": int(st1["image_bytes"] > st0["image_bytes"]),
                            "rebuilds": st1["rebuilds"] - st0["rebuilds"],
                            "broadcast_ms_per_batch": acc["delta"] * 1e3 / args.steps if sync else None,
                            "headroom_vs_100k_per_s": (ops_n / (host_ns / 1e9)) / 1e5 if host_ns else None},
            "match_batches_per_delta_batch": per_period,
            "pairs_per_s": emitted * args.steps * per_period * world / t_max,
            "emissions_per_match_batch": emitted, "load_s": load_s,
            "verified": {"known_answer": known, "replicas_equal": replicas_equal, "images_equal": images_equal},
            "kernel_us": stages,
            "served": {"deferred": st1["deferred_tier1"], "retried": st1["retried"],
                       "many_key": st1["many_key"], "wave_entries": wave_rec, "wide_entries": st1["wide_entries"],
                       "dedup": st1["dedup"], "dedup_walked": st1["dedup_walked"]},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": achieved / PEAK_HBM_GBS if achieved else None,
                         "traffic": d_traffic,
                         # no physical frac here: the counters' bytes include
                         # the alarm lists re-fetched per publish (waste, not
                         # work); traffic / algorithmic bytes says how much
                         "traffic_over_compulsory": d_traffic / alg_emit if d_traffic and alg_emit else None,
                         "kernel": dom["kernel"], "algorithmic_bytes_per_launch": alg_emit,
                         "bytes_model": "16 B written per record this launch writes (compulsory lower bound)",
                         "per_kernel": per_kernel, "step_level": step_level,
                         "survey_model_achieved_step": 32 * emitted / (stages["per_call"] * 1e3)
                         if stages["per_call"] else None},
            "survey_bytes_per_publish": b_p,
            "count_kernel": {"us": count_ns / 1e3,
                             "achieved": (b_p["lookup"] * npub / count_ns) if (b_p and count_ns) else None,
                             "bytes_model": "8(L+1) + 16 S_p per publish, S_p from the oracle's lookup counters on "
                                            "256 publishes"},
            "cpu_baseline": cpu,
            "arena_bytes": st1["device_bytes"],
            "deferred": [st1["deferred_tier1"], st1["deferred_tier2"]],
            "build_id": _lib.build_id(),
        }
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


def bench_retain(args):
    """Retained-message matching (vmq_retain_srv:match_fold/4, SURVEY §8(f)
    rank 3): 1M retained topics, one step = one burst of 2^18 subscription
    filters folded over the store on one GPU (plan, chunk count, scan, emit
    of message ids).  Prints one JSON line with the walk kernel's roofline
    and the CPU restatement (a full ets:foldl per wildcard filter, as the
    reference) timed on a bounded sample."""
    import torch
    from vernemq_amd import workloads as W
    from vernemq_amd.retain import RetainGpuSrv
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t0 = time.time()
    w = W.RetainWorkload(n_dev=args.rt_devices, n_filters=args.rt_filters, n_heavy=args.rt_heavy)
    srv = RetainGpuSrv(device=0, hint_topics=w.n_topics)
    vid = w.load_into(srv)
    load_s = time.time() - t0
    log("RT: %d retained topics loaded in %.1fs, %s" % (w.n_topics, load_s, srv.stats_raw()))
    arr, words = w.filter_arrays(vid)
    nf = len(arr)
    d_f = torch.from_numpy(arr.view(np.uint32).reshape(-1).copy()).to(dev)
    d_w = torch.from_numpy(words.astype(np.int32)).to(dev)
    total = int(w.matches.sum())
    out_cap = total + 1024
    d_o = torch.empty(out_cap, dtype=torch.int32, device=dev)
    d_offs = torch.zeros(nf + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    step = lambda: srv.match_device(d_f.data_ptr(), nf, d_w.data_ptr(), d_o.data_ptr(), out_cap,
                                    d_offs.data_ptr(), sp)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    rc = srv.match_status(sp)
    if rc != 0:
        raise RuntimeError("retain match status %d after warmup" % rc)
    # size-independent check: per-filter match counts = the workload's known answer,
    # and every emitted message id's topic matches its filter (sampled)
    offs = d_offs.cpu().numpy()
    verified = bool(np.array_equal(np.diff(offs), w.matches))
    if not verified:
        raise RuntimeError("per-filter retained match counts differ from the workload's known answer")
    srv.set_timing(not args.no_timing)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    rc = srv.match_status(sp)
    if rc != 0:
        raise RuntimeError("retain match status %d in timed region" % rc)
    count_ns, emit_ns, nl = srv.kernel_times()
    alg = w.algorithmic_bytes("walk")
    achieved = alg / emit_ns if emit_ns else None

    cpu = None
    if not args.no_cpu_baseline:
        from oracle import retain_oracle as RO   # the CPU restatement: baseline only
        t0 = time.time()
        orc = RO.RetainOracle()
        B = 1 << 17
        for lo in range(0, w.n_topics, B):
            orc.apply([("insert", "", w.topic(i), i) for i in range(lo, min(w.n_topics, lo + B))])
        log("RT cpu baseline: oracle loaded in %.1fs" % (time.time() - t0))
        S = 64
        sample = [("", w.filter(i)) for i in range(S)]
        ns1, _ = orc.match_timed(sample, 1)
        reps = max(1, int(math.ceil(args.cpu_seconds * 1e9 / max(ns1, 1))))
        ns, _ = orc.match_timed(sample, reps)
        cpu = {"value": S * reps / (ns / 1e9), "unit": "filters/s", "cores": 1, "kind": "port",
               "sample": "first %d filters of the RT batch x %d reps (%.1fs), 1 thread, oracle/vmq_retain_oracle.cpp "
                         "(C++ restatement of vmq_retain_srv:match_fold/4: ets:lookup for exact filters, a full "
                         "ets:foldl + vmq_topic:match/2 per wildcard filter; not BEAM); host %s"
                         % (S, reps, ns / 1e9, cpu_model())}
        log("RT cpu baseline: %.0f filters/s" % cpu["value"])

    st = srv.stats_raw()
    print(json.dumps({
        "metric": "retained match_fold: subscription filters matched/sec (1M retained topics)",
        "value": nf * args.steps / el, "unit": "filters/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: vernemq_amd.workloads.RetainWorkload (splitmix64 seed 0x7E7)",
        "config": {"workload": "RT: %d retained devices/{d}/telemetry/{m}; %d filters/step (50%% d/telemetry/#, "
                               "20%% d/+/m, 25%% exact, 5%% unknown device, %d x devices/+/telemetry/m)"
                               % (w.n_topics, nf, w.n_heavy)},
        "messages_per_s": total * args.steps / el, "matches_per_step": total,
        "verified_counts": verified,
        "kernel_us": {"plan_scan": count_ns / 1e3, "walk": emit_ns / 1e3, "launches": nl},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS if achieved else None,
                     "traffic": load_pmc_traffic("k_rt_walk", "pmc_rt.json"),
                     "kernel": "k_rt_walk (one-pass walk + emit)", "algorithmic_bytes_per_launch": alg,
                     "bytes_model": "32 B per visited candidate (its list entry) + 4 B per match + "
                                    "40 B per filter (workloads.RetainWorkload.algorithmic_bytes)"},
        "cpu_baseline": cpu, "load_s": load_s, "arena_bytes": st["device_bytes"],
        "partitions": st["partitions"]}), flush=True)


def bench_acl(args):
    """ACL checks (vmq_acl:check/4 via auth_on_publish / auth_on_subscribe,
    SURVEY §8(f) rank 4): 2^20 checks per step of config C's device fleet
    against an ACL of 64 `all` rules, 15,625 users x 4 rules and 8 patterns
    (vernemq_amd.workloads.AclWorkload).  Prints one JSON line with the
    check kernel's roofline and the CPU restatement timed on a sample."""
    import torch
    from vernemq_amd import workloads as W
    from vernemq_amd.acl import AclGpu
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t0 = time.time()
    w = W.AclWorkload(n_reqs=args.ac_requests)
    acl = AclGpu(device=0)
    lines = w.lines()
    acl.load_from_list(lines)
    reqs, words = w.arrays(acl)
    load_s = time.time() - t0
    log("AC: ACL of %d lines loaded in %.1fs, %s" % (len(lines), load_s, acl.stats_raw()))
    n = len(reqs)
    d_r = torch.from_numpy(reqs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_w = torch.from_numpy(words.astype(np.int32)).to(dev)
    d_o = torch.zeros(n, dtype=torch.uint8, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    step = lambda: acl.check_device(d_r.data_ptr(), n, d_w.data_ptr(), d_o.data_ptr(), sp)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    rc = acl.check_status(sp)
    if rc != 0:
        raise RuntimeError("acl check status %d after warmup" % rc)
    verified = bool(np.array_equal(d_o.cpu().numpy(), w.expect))   # the workload's known answer
    if not verified:
        raise RuntimeError("ACL verdicts differ from the workload's known answer")
    acl.set_timing(not args.no_timing)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    rc = acl.check_status(sp)
    if rc != 0:
        raise RuntimeError("acl check status %d in timed region" % rc)
    check_ns, nl = acl.kernel_times()
    alg = w.algorithmic_bytes()
    achieved = alg / check_ns if check_ns else None

    cpu = None
    if not args.no_cpu_baseline:
        from oracle import acl_oracle as AO   # the CPU restatement: baseline only
        orc = AO.AclOracle()
        orc.load_from_list(lines)
        S = 20_000
        sample = [w.request(i) for i in range(S)]
        ns1, _ = orc.check_timed(sample, 1)
        reps = max(1, int(math.ceil(args.cpu_seconds * 1e9 / max(ns1, 1))))
        ns, _ = orc.check_timed(sample, reps)
        cpu = {"value": S * reps / (ns / 1e9), "unit": "checks/s", "cores": 1, "kind": "port",
               "sample": "first %d requests of the AC batch x %d reps (%.1fs), 1 thread, oracle/vmq_acl_oracle.cpp "
                         "(C++ restatement of vmq_acl:check/4: all -> user -> pattern lists, vmq_topic:match/2 per "
                         "rule; not BEAM); host %s" % (S, reps, ns / 1e9, cpu_model())}
        log("AC cpu baseline: %.0f checks/s" % cpu["value"])

    st = acl.stats_raw()
    print(json.dumps({
        "metric": "ACL checks/sec (vmq_acl auth_on_publish / auth_on_subscribe)",
        "value": n * args.steps / el, "unit": "checks/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: vernemq_amd.workloads.AclWorkload (splitmix64 seed 0xAC)",
        "config": {"workload": "AC: %d checks/step (80%% allowed publishes via pattern %%c, 10%% denied, 5%% "
                               "subscribes, 5%% user-table publishes); ACL %d rules, %d users"
                               % (n, st["rules"], st["users"])},
        "verified_counts": verified,
        "kernel_us": {"check": check_ns / 1e3, "launches": nl},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS if achieved else None,
                     "traffic": load_pmc_traffic("k_acl_check", "pmc_ac.json"),
                     "kernel": "k_acl_check", "algorithmic_bytes_per_launch": alg,
                     "bytes_model": "24-B request + 16-B topic words read, 1-B verdict written per check "
                                    "(the rule tables are L2-resident; workloads.AclWorkload.algorithmic_bytes)"},
        "cpu_baseline": cpu, "load_s": load_s, "arena_bytes": st["device_bytes"]}), flush=True)


def bench_shared(args):
    """Shared-subscription dispatch (vmq_shared_subscriptions:publish/3,
    SURVEY §8(f) rank 4) on config D's match output: the 2^20-publish batch
    is matched once on the device (untimed; its records stay in HBM), then
    each step dispatches the whole batch with the default prefer_local policy
    (every $share group of every publish gets its member; queue states: 3/4
    online, 1/8 offline, 1/16 draining, 1/16 no queue).  Prints one JSON line
    with the dispatch kernels' roofline and the CPU restatement on a sample."""
    import torch
    from vernemq_amd import workloads as W
    from vernemq_amd.reg_view import RegGpuView
    from vernemq_amd.shared import SharedGpu
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t0 = time.time()
    w = W.config_d(scale=args.d_scale, n_pubs=args.batch)
    n_live = w.notes["n_live"]
    view = RegGpuView(node=w.self_node, device=0, nodes=w.nodes,
                      hints={"edges": 4 * n_live // 5, "paths": 4 * n_live // 5, "keys": n_live,
                             "records": n_live * 11 // 10, "exact": n_live})
    w.load_into(view, n=n_live)
    load_s = time.time() - t0
    log("SS: config D (%d live subs) loaded in %.1fs" % (n_live, load_s))
    pubs, words = w.publish_arrays(view)
    npub = len(pubs)
    d_pubs = torch.from_numpy(pubs.view(np.uint32).reshape(-1).copy()).to(dev)
    d_words = torch.from_numpy(words.astype(np.int32)).to(dev)
    d_offs = torch.zeros(npub + 1, dtype=torch.int64, device=dev)
    sp = torch.cuda.current_stream().cuda_stream
    out_cap = 1024
    d_out = torch.empty(4, dtype=torch.int32, device=dev)
    for _ in range(2):   # first pass sizes the output
        view.match_device(d_pubs.data_ptr(), npub, d_words.data_ptr(), d_out.data_ptr(), out_cap,
                          d_offs.data_ptr(), sp)
        torch.cuda.synchronize()
        need = int(d_offs[-1].item())
        rc = view.match_status(sp)
        if need <= out_cap and rc == 0:
            break
        out_cap = need + 1024
        d_out = torch.empty(out_cap * 4, dtype=torch.int32, device=dev)
    total = int(d_offs[-1].item())
    sel = SharedGpu(device=0, local_node=0)
    n_sub = len(w.clients)
    st = np.ones(n_sub, dtype=np.uint8)
    u = W.SplitMix(0x55).ints(n_sub, 16)
    st[u >= 12] = 2   # offline
    st[u == 14] = 3   # draining
    st[u == 15] = 0   # no queue
    ids = np.array([view.subscribers.ids[c] for c in w.clients], dtype=np.uint32)
    sel.set_state_ids(ids, st)
    d_ch = torch.empty(total, dtype=torch.uint8, device=dev)
    d_f = torch.empty(npub, dtype=torch.int32, device=dev)
    step = lambda k: sel.select_device(d_out.data_ptr(), d_offs.data_ptr(), npub, "prefer_local", 0x55, k * npub,
                                       d_ch.data_ptr(), d_f.data_ptr(), sp)
    n_warm = max(1, args.warmup)
    for k in range(n_warm):
        step(k)
    torch.cuda.synchronize()
    if sel.select_status(sp) != 0:
        raise RuntimeError("select status after warmup")
    # parity on a sample of the batch against the CPU restatement
    from oracle import shared_oracle as SO   # checker (and CPU baseline) only
    offs_h = d_offs.cpu().numpy().astype(np.uint64)
    S = min(npub, 65536)
    recs_s = d_out[: int(offs_h[S]) * 4].cpu().numpy().view(np.uint32).reshape(-1, 4)
    full_states = np.ones(int(ids.max()) + 1, np.uint8)
    full_states[ids] = st
    k_last = n_warm - 1
    want_c, want_f = SO.select(recs_s, offs_h[: S + 1], "prefer_local", 0x55, k_last * npub, full_states, 0)
    got_c = d_ch[: int(offs_h[S])].cpu().numpy()
    got_f = d_f[:S].cpu().numpy().astype(np.uint32)
    verified = bool(np.array_equal(got_c, want_c) and np.array_equal(got_f, want_f))
    if not verified:
        raise RuntimeError("dispatch differs from the CPU restatement on the sample")
    n_group = int((recs_s[:, 0] >> 24 == 2).sum())
    sel.set_timing(not args.no_timing)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(n_warm + k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if sel.select_status(sp) != 0:
        raise RuntimeError("select status in timed region")
    sel_ns, nl, deferred = sel.kernel_times()
    alg = total * 17 + npub * 12   # per record: 16-B read + 1-B chosen; per publish: offsets + failed
    achieved = alg / sel_ns if sel_ns else None
    chosen_n = int(d_ch.sum().item())

    cpu = None
    if not args.no_cpu_baseline:
        thr = {}
        for threads in (1, args.cpu_threads):
            s1 = SO.select_timed(recs_s, offs_h[: S + 1], "prefer_local", 0x55, full_states, 0, 1, threads)
            reps = max(1, int(math.ceil(args.cpu_seconds / max(s1, 1e-6))))
            sec = SO.select_timed(recs_s, offs_h[: S + 1], "prefer_local", 0x55, full_states, 0, reps, threads)
            thr[threads] = (S * reps / sec, reps, sec)
        v, reps, sec = thr[args.cpu_threads]
        cpu = {"value": v, "unit": "publishes/s", "cores": args.cpu_threads, "kind": "port",
               "single_thread_value": thr[1][0],
               "sample": "first %d publishes of the SS batch (%d records) x %d reps (%.1fs) on %d threads "
                         "(1 thread: %.3g publishes/s), oracle/vmq_shared_oracle.cpp (C++ restatement of "
                         "add_to_subscriber_group + vmq_shared_subscriptions:publish/3: group map, "
                         "filter_subscribers, keyed sort, publish_online / publish_any; not BEAM); host %s"
                         % (S, len(recs_s), reps, sec, args.cpu_threads, thr[1][0], cpu_model())}
        log("SS cpu baseline: %.0f publishes/s (%d threads), %.0f (1 thread)" % (v, args.cpu_threads, thr[1][0]))

    print(json.dumps({
        "metric": "shared-subscription dispatches/sec (publishes through vmq_shared_subscriptions:publish/3)",
        "value": npub * args.steps / el, "unit": "publishes/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": el * 1e3 / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic: SURVEY.md §8(d) config D generator (splitmix64 seed 0xD), scale %g" % args.d_scale,
        "config": {"workload": "SS: config D match output, %d publishes / %d records per step (%d $share records "
                               "in the first %d publishes), policy prefer_local" % (npub, total, n_group, S)},
        "verified_sample": verified, "records_per_step": total, "chosen_per_step": chosen_n,
        "kernel_us": {"select": sel_ns / 1e3, "launches": nl, "tier2_publishes": deferred},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS if achieved else None,
                     "traffic": load_pmc_traffic("k_select_wave", "pmc_ss.json"),
                     "kernel": "k_select_wave + k_select_block",
                     "note": "byte-bound by HBM in principle (one read of the records); measured at ~36 % of peak "
                             "it is limited by per-wave latency (load -> LDS claim -> reduction -> write phases)",
                     "algorithmic_bytes_per_launch": alg,
                     "bytes_model": "16-B record read + 1-B chosen written per record, 8-B offset + 4-B failed "
                                    "per publish (queue states are L2-resident)"},
        "cpu_baseline": cpu, "load_s": load_s}), flush=True)


if __name__ == "__main__":
    sys.exit(main() or 0)
