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
