"""Multi-GPU replication of the matcher tables over ``torch.distributed``
(RCCL over xGMI on MI355X; gloo for the CPU tests).

The path shards by publish: every GPU holds a full replica of
the tables and matches its own publish batches; the only collectives are

* the device image broadcast when a replica starts or the primary re-lays
  its arena out (``ImageSync.full``),
* the 24-B patch records of each delta batch (``ImageSync.delta``) plus the
  256-B layout (its trie depth sizes the wave tier's stack) — rank 0 runs
  the host engine (``vmqg_apply_ops``), every rank applies the same bytes, so
  all replicas stay byte-identical at each epoch,
* an all-gather of per-GPU counts (``gather_counts``).

Nothing on the match data path is communicated.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def shard(n: int, rank: int, world: int):
    """Contiguous [lo, hi) share of n items for `rank` (publish sharding)."""
    return n * rank // world, n * (rank + 1) // world


def _comm_device(dist, device, group=None):
    """Where collective buffers live: the GPU for nccl (RCCL over xGMI),
    host memory for gloo (CPU tests, or a one-GPU rehearsal of N ranks)."""
    import torch
    if dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return device


def _bcast_bytes(dist, data, src: int, device, group=None):
    """Broadcast a byte string (given on src) -> uint8 tensor on `device`."""
    import torch
    cdev = _comm_device(dist, device, group)
    n = torch.zeros(1, dtype=torch.int64, device=cdev)
    if dist.get_rank(group) == src:
        n[0] = len(data)
    dist.broadcast(n, src, group=group)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=cdev)
    if dist.get_rank(group) == src and len(data):
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    if buf.numel():
        dist.broadcast(buf, src, group=group)
    return buf.to(device)


def gather_counts(dist, values, device, group=None):
    """All-gather a small int64 vector from every rank -> [world, k] array."""
    import torch
    t = torch.as_tensor(np.asarray(values, dtype=np.int64), device=_comm_device(dist, device, group))
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return np.stack([o.cpu().numpy() for o in out])


class ImageSync:
    """Primary (rank `src`, a RegGpuView with the host engine) -> replicas.

    GPU mode (`device` is a cuda device): replicas are RegGpuView contexts
    created with replica=True; images and patches land directly in their
    device arenas.  Host mode (`device` is cpu, used by the gloo tests): the
    replica side keeps a numpy image and applies patches itself, so the tests
    can prove that the patch stream reproduces the primary's image bytes.
    """

    def __init__(self, dist, view, device, src: int = 0, group=None):
        self.dist, self.view, self.device, self.src, self.group = dist, view, device, src, group
        self.rank = dist.get_rank(group)
        self.image = None     # host mode replica image
        self.layout = None

    @property
    def primary(self) -> bool:
        return self.rank == self.src

    def _gpu(self) -> bool:
        return getattr(self.device, "type", str(self.device)) != "cpu"

    def full(self):
        """Broadcast the primary's whole image; replicas adopt it."""
        import torch
        d = self.dist
        if self.primary:
            ptr, nbytes, lay = self.view.arena()
        else:
            ptr, nbytes, lay = 0, 0, b""
        lay_t = _bcast_bytes(d, lay, self.src, self.device, self.group)
        cdev = _comm_device(d, self.device, self.group)
        n = torch.tensor([nbytes], dtype=torch.int64, device=cdev)
        d.broadcast(n, self.src, group=self.group)
        nbytes = int(n.item())
        img = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        if self.primary:
            if self._gpu():
                hip_memcpy_d2d(img.data_ptr(), ptr, nbytes)
            else:
                img.copy_(torch.from_numpy(self.view.export_image()))
        if self._gpu():
            torch.cuda.synchronize(self.device)
        if cdev.type == "cpu" and self._gpu():   # gloo rehearsal: stage through host memory
            host = img.cpu()
            d.broadcast(host, self.src, group=self.group)
            img.copy_(host)
        else:
            d.broadcast(img, self.src, group=self.group)
        self.layout = bytes(lay_t.cpu().numpy())
        if not self.primary:
            if self._gpu():
                self.view.replica_load(self.layout, img.data_ptr())
                torch.cuda.synchronize(self.device)
            else:
                self.image = img.numpy().copy()
        return nbytes

    def delta(self):
        """After the primary applied a batch: ship its patches (or the full
        image when the batch re-laid the arena out)."""
        import torch
        d = self.dist
        flag = torch.zeros(1, dtype=torch.int64, device=_comm_device(d, self.device, self.group))
        data, lay = b"", b""
        if self.primary:
            data, full = self.view.last_patches()
            flag[0] = 1 if full else 0
            lay = self.view.arena()[2]
        d.broadcast(flag, self.src, group=self.group)
        if int(flag.item()):
            self.full()
            return -1
        lay_t = _bcast_bytes(d, lay, self.src, self.device, self.group)
        buf = _bcast_bytes(d, data, self.src, self.device, self.group)
        if not self.primary:
            self.layout = bytes(lay_t.cpu().numpy())
            if self._gpu():
                self.view.replica_sync_layout(self.layout)
                if buf.numel():
                    self.view.apply_patches_device(buf.data_ptr(), buf.numel())
                torch.cuda.synchronize(self.device)
            elif buf.numel():
                apply_patches_host(self.image, buf.numpy())
        return buf.numel() // 24


PATCH_DTYPE = np.dtype([("off", "<u8"), ("data", "<u4", (4,))])


def apply_patches_host(image: np.ndarray, patches: np.ndarray):
    """numpy restatement of k_apply_patches (16-B stores at 16-B offsets)."""
    p = np.frombuffer(np.ascontiguousarray(patches).tobytes(), dtype=PATCH_DTYPE)
    if len(p):
        img32 = image.view(np.uint32)
        idx = (p["off"] // 4).astype(np.int64)
        for j in range(4):
            img32[idx + j] = p["data"][:, j]


def hip_memcpy_d2d(dst: int, src: int, n: int):
    """Device-to-device copy through the process's one HIP runtime: the
    hipMemcpy libvmqgpu itself resolves (its DT_NEEDED libamdhip64.so.7,
    torch's copy once torch is imported) — never a second runtime loaded by
    a bare "libamdhip64.so"."""
    import ctypes
    hip_memcpy = _lib.lib().hipMemcpy   # dlsym through libvmqgpu's dependencies
    hip_memcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    hip_memcpy.restype = ctypes.c_int
    rc = hip_memcpy(dst, src, n, 3)
    if rc != 0:
        raise _lib.VmqgError(_lib.E_DEVICE, "hipMemcpy D2D (%d)" % rc)
