"""Multi-GPU replication of the matcher tables over ``torch.distributed``
(RCCL over xGMI on MI355X; gloo for the CPU tests).

The path shards by publish: every GPU holds a full replica of
the tables and matches its own publish batches; the only collectives are

* the device image broadcast when a replica starts or the primary re-lays
  its arena out (``ImageSync.full``),
* the 24-B patch records of each delta batch (``ImageSync.delta``) — rank 0
  runs the host engine (``vmqg_apply_ops``), every rank applies the same
  bytes, so all replicas stay byte-identical at each epoch; sizes and the
  256-B layout (its trie depth sizes the wave tier's stack) go over a
  host-side gloo group, so the delta path never waits on a GPU stream,
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


def gather_counts(dist, values, device, group=None):
    """All-gather a small int64 vector from every rank -> [world, k] array."""
    import torch
    t = torch.as_tensor(np.array(values, dtype=np.int64), device=_comm_device(dist, device, group))   # a copy: callers may pass read-only views
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(out, t, group=group)
    return np.stack([o.cpu().numpy() for o in out])


class ImageSync:
    """Primary (rank `src`, a RegGpuView with the host engine) -> replicas.

    GPU mode (`device` is a cuda device): replicas are RegGpuView contexts
    created with replica=True; images and patches land directly in their
    device arenas, stream-ordered behind the matches already queued (no
    device synchronisation on the delta path).  The small control messages
    (image / patch sizes, the full-image flag, the 256-B layout) travel over
    a host-side gloo group, so no rank has to read a GPU tensor back to learn
    a size; the payloads travel over `group` (RCCL over xGMI with nccl).
    Host mode (`device` is cpu, used by the gloo tests): the replica side
    keeps a numpy image and applies patches itself, so the tests can prove
    that the patch stream reproduces the primary's image bytes.
    """

    def __init__(self, dist, view, device, src: int = 0, group=None, ctrl_group=None):
        self.dist, self.view, self.device, self.src, self.group = dist, view, device, src, group
        self.rank = dist.get_rank(group)
        if ctrl_group is None:
            ctrl_group = group if dist.get_backend(group) == "gloo" else dist.new_group(backend="gloo")
        self.ctrl = ctrl_group
        self.image = None     # host mode replica image
        self.layout = None
        self._stream = None   # GPU replicas: where images and patches land (see _side_stream)

    @property
    def primary(self) -> bool:
        return self.rank == self.src

    def _gpu(self) -> bool:
        return getattr(self.device, "type", str(self.device)) != "cpu"

    def _ctrl(self, values, layout: bytes = b""):
        """Broadcast a few int64s and the layout bytes over the host group."""
        import torch
        t = torch.zeros(len(values) + 1 + 32, dtype=torch.int64)
        if self.primary:
            t[: len(values)] = torch.tensor(values, dtype=torch.int64)
            t[len(values)] = len(layout)
            if layout:
                t[len(values) + 1:len(values) + 1 + len(layout) // 8] = torch.frombuffer(bytearray(layout),
                                                                                     dtype=torch.int64)
        self.dist.broadcast(t, self.src, group=self.ctrl)
        vals = [int(x) for x in t[: len(values)]]
        nl = int(t[len(values)])
        lay = t[len(values) + 1:len(values) + 1 + nl // 8].numpy().tobytes() if nl else b""
        return vals, lay

    def _side_stream(self, buf):
        """A stream of its own for the library's image / patch copy, after
        everything queued on torch's current stream (the payload's broadcast
        or host staging).  Never pass torch's default stream through: its
        handle is 0, which the library reads as "my context stream", a
        different stream that would not wait for the payload.  `buf` stays
        allocated until the side stream has used it."""
        import torch
        if self._stream is None:
            self._stream = torch.cuda.Stream(self.device)
        self._stream.wait_stream(torch.cuda.current_stream(self.device))
        buf.record_stream(self._stream)
        return self._stream

    def _payload(self, nbytes: int, fill=None):
        """A uint8 device tensor of nbytes broadcast from the primary
        (`fill(tensor)` writes the primary's bytes)."""
        import torch
        cdev = _comm_device(self.dist, self.device, self.group)
        buf = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        if self.primary and fill is not None and nbytes:
            fill(buf)
        if not nbytes:
            return buf
        if cdev.type == "cpu" and self._gpu():   # gloo rehearsal: stage through host memory
            host = buf.cpu()
            self.dist.broadcast(host, self.src, group=self.group)
            buf.copy_(host, non_blocking=True)
        else:
            self.dist.broadcast(buf, self.src, group=self.group)
        return buf

    def full(self):
        """Broadcast the primary's whole image; replicas adopt it."""
        import torch
        if self.primary:
            ptr, nbytes, lay = self.view.arena()
        else:
            ptr, nbytes, lay = 0, 0, b""
        (nbytes,), lay = self._ctrl([nbytes], lay)
        self.layout = lay

        def fill(buf):
            if self._gpu():
                torch.cuda.synchronize(self.device)   # the primary's arena is up to date
                hip_memcpy_d2d(buf.data_ptr(), ptr, nbytes)
            else:
                buf.copy_(torch.from_numpy(self.view.export_image()))

        img = self._payload(nbytes, fill)
        if not self.primary:
            if self._gpu():
                st = self._side_stream(img)
                self.view.replica_load(self.layout, img.data_ptr(), st.cuda_stream)
                torch.cuda.synchronize(self.device)   # img is released after the copy
            else:
                self.image = img.numpy().copy()
        return nbytes

    def delta(self):
        """After the primary applied a batch: ship its patches (or the full
        image when the batch re-laid the arena out).  Returns the number of
        patch records (-1: a full image was shipped)."""
        import torch
        data, full, lay = b"", 0, b""
        if self.primary:
            data, f = self.view.last_patches()
            full = 1 if f else 0
            lay = self.view.arena()[2]
        (full, nbytes), lay = self._ctrl([full, len(data)], lay)
        if full:
            self.full()
            return -1

        def fill(buf):
            buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8), non_blocking=False)

        buf = self._payload(nbytes, fill)
        if not self.primary:
            self.layout = lay
            if self._gpu():
                self.view.replica_sync_layout(lay)
                if nbytes:
                    st = self._side_stream(buf)
                    self.view.apply_patches_device(buf.data_ptr(), nbytes, st.cuda_stream)
            elif nbytes:
                apply_patches_host(self.image, buf.numpy())
        return nbytes // 24


REGION_NAMES = ("edges", "nodes", "keydesc", "keylist", "records", "exact", "exwords")


def arena_region_hashes(view, device):
    """64-bit hashes of the seven arena regions of a view's device image
    (the layout's region offsets), to compare replicas with the primary."""
    import hashlib

    import torch
    ptr, nbytes, lay = view.arena()
    torch.cuda.synchronize(device)
    img = torch.empty(nbytes, dtype=torch.uint8, device=device)
    hip_memcpy_d2d(img.data_ptr(), ptr, nbytes)
    host = img.cpu().numpy()
    offs = [int(x) for x in np.frombuffer(lay[16:72], dtype=np.uint64)] + [nbytes]
    return [int.from_bytes(hashlib.sha256(host[offs[i]:offs[i + 1]].tobytes()).digest()[:8], "little", signed=True)
            for i in range(len(REGION_NAMES))]


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
