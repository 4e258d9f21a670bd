"""World-size-2 tests of the multi-GPU replication protocol on CPU (gloo):
rank 0 runs the host engine; rank 1 follows by the broadcast image + the
patch stream and must hold a byte-identical image after every delta batch —
the same bytes RCCL carries between MI355X ranks in bench.py."""
import hashlib
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, seed):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tests import harness as H
    from vernemq_amd import dist as vd
    from vernemq_amd.reg_view import RegGpuView
    dev = torch.device("cpu")
    wl = H.ChurnWorkload(seed, n_clients=80)
    view = RegGpuView(node=wl.self_node, device=-1) if rank == 0 else None
    sync = vd.ImageSync(dist, view, dev)
    if rank == 0:
        view.handle_events([wl.event() for _ in range(50)])
    sync.full()
    log = []
    for step in range(12):
        if rank == 0:
            view.handle_events([wl.event() for _ in range(30)])
        n = sync.delta()
        if rank == 0:
            img = view.export_image()
        else:
            img = sync.image
        h = hashlib.sha256(img.tobytes()).digest()
        hv = np.frombuffer(h[:16], dtype=np.int64)
        allh = vd.gather_counts(dist, hv, dev)
        log.append((n, bool((allh[0] == allh[1]).all())))
    # publish sharding + count all-gather
    lo, hi = vd.shard(1000, rank, world)
    cnt = vd.gather_counts(dist, [hi - lo, rank], dev)
    if rank == 0:
        with open(os.path.join(out_dir, "result.txt"), "w") as f:
            f.write(repr({"log": log, "counts": cnt.tolist()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_image_and_patch_replication(tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path), 5), nprocs=2, join=True)
    res = eval(open(tmp_path / "result.txt").read())
    assert all(same for _, same in res["log"]), res["log"]
    assert any(n > 0 for n, _ in res["log"])            # patches were shipped
    assert res["counts"] == [[500, 0], [500, 1]]


def test_shard_covers_range():
    from vernemq_amd.dist import shard
    for n in (0, 1, 7, 1 << 20):
        for w in (1, 2, 3, 8):
            parts = [shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))


def test_host_patch_apply_matches_mirror():
    """Single process: image + patches reproduce the next image exactly."""
    from tests import harness as H
    from vernemq_amd import dist as vd
    from vernemq_amd.reg_view import RegGpuView
    wl = H.ChurnWorkload(11)
    v = RegGpuView(node=wl.self_node, device=-1)
    v.handle_events([wl.event() for _ in range(40)])
    img = v.export_image()
    for _ in range(10):
        v.handle_events([wl.event() for _ in range(15)])
        data, full = v.last_patches()
        if full:
            img = v.export_image()
            continue
        vd.apply_patches_host(img, np.frombuffer(data, dtype=np.uint8))
        assert np.array_equal(img, v.export_image())


def _gpu_worker(rank, world, port, out_dir, seed):
    """Both ranks on cuda:0 over gloo (the same ImageSync code that runs over
    RCCL in bench.py): rank 0 owns the host engine, rank 1 a replica fed by
    the image + patch stream; after every churn batch both match the same
    publishes and must agree byte for byte (and rank 0 with the oracle)."""
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from oracle import oracle as O
    from tests import harness as H
    from vernemq_amd import dist as vd
    from vernemq_amd.reg_view import EMIT_DTYPE, PUB_DTYPE, RegGpuView
    wl = H.ChurnWorkload(seed, n_clients=80)
    if rank == 0:
        view = RegGpuView(node=wl.self_node, device=0, nodes=wl.nodes)
        orc = O.TrieOracle(wl.self_node)
        evs = [wl.event() for _ in range(60)]
        view.handle_events(evs)
        orc.apply(evs)
    else:
        view = RegGpuView(node=wl.self_node, device=0, replica=True)
    sync = vd.ImageSync(dist, view, dev)
    sync.full()
    log = []
    for step in range(10):
        if rank == 0:
            evs = [wl.event() for _ in range(25)]
            view.handle_events(evs)
            orc.apply(evs)
        n = sync.delta()
        # rank 0 prepares the batch (it owns the dictionary), both match it
        if rank == 0:
            pubs = wl.publishes(150)
            arr, words = view.prepare(pubs)
            hdr = torch.tensor([len(arr), len(words)], dtype=torch.int64)
        else:
            hdr = torch.zeros(2, dtype=torch.int64)
        dist.broadcast(hdr, 0)
        a_t = torch.from_numpy(arr.view(np.uint32).view(np.int32).copy()) if rank == 0 else \
            torch.zeros(int(hdr[0]) * 4, dtype=torch.int32)
        w_t = torch.from_numpy(words.astype(np.int32)) if rank == 0 else torch.zeros(int(hdr[1]), dtype=torch.int32)
        dist.broadcast(a_t, 0)
        dist.broadcast(w_t, 0)
        arr_r = a_t.numpy().view(np.uint32).view(PUB_DTYPE)
        recs, offs = view.match_arrays(arr_r, w_t.numpy().view(np.uint32))
        h = hashlib.sha256(offs.tobytes() + recs.view(EMIT_DTYPE).tobytes()).digest()
        allh = vd.gather_counts(dist, np.frombuffer(h[:16], dtype=np.int64), dev)
        oracle_ok = True
        if rank == 0:
            want = orc.fold_batch([(mp, b"pub", t) for mp, t in pubs])
            got = [sorted(H.canon(view.decode(recs[j])) for j in range(int(offs[i]), int(offs[i + 1])))
                   for i in range(len(pubs))]
            oracle_ok = all(g == sorted(x) for g, x in zip(got, want))
        log.append((n, bool((allh[0] == allh[1]).all()), oracle_ok, int(offs[-1])))
    if rank == 0:
        with open(os.path.join(out_dir, "gpu_result.txt"), "w") as f:
            f.write(repr(log))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_rank_replica_matches_equal_primary_under_churn(tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.spawn(_gpu_worker, args=(2, port, str(tmp_path), 9), nprocs=2, join=True)
    log = eval(open(tmp_path / "gpu_result.txt").read())
    assert all(same for _, same, _, _ in log), log
    assert all(ok for _, _, ok, _ in log), log
    assert any(n > 0 for n, _, _, _ in log)           # patches were shipped
    assert sum(e for _, _, _, e in log) > 100          # the publishes do match
