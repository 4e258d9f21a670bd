#!/usr/bin/env python3
"""Compile libvmqgpu.so variants for A/B runs (tools/rt_ab.sh): the same
sources and flags as vernemq_amd._lib.build plus -D knobs, into build/ab/."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vernemq_amd import _lib  # noqa: E402

VARIANTS = {
    "default": [],
    "tail8": ["-DVMQG_TAIL_BPC=8"],
    "walkcall": ["-DVMQG_WALK_CALL=1"],
    "wide32": ["-DVMQG_WIDE_LANES=32"],
    "recwide256": ["-DVMQG_WIDE_RECORDS=256"],
    "nofilter": ["-DVMQG_EXACT_FILTER=0"],
    "nowalk": ["-DVMQG_TAIL_NOWALK=1"],
    "nowalk_u16": ["-DVMQG_TAIL_NOWALK=1", "-DVMQG_TAIL_U=16"],
    "tail_u4": ["-DVMQG_TAIL_U=4"],
    "count_wpe5": ["-DVMQG_COUNT_WPE=5"],
    "nospill": ["-DVMQG_SPILL_KEYS=2"],
    "noalias": ["-DVMQG_HASH_ALIAS=0"],
    "scan4": ["-DVMQG_SCAN_ITEMS=4"],
    "scan8": ["-DVMQG_SCAN_ITEMS=8"],
    "emit_u2": ["-DVMQG_EMIT_U=2"],
    "emit_u8": ["-DVMQG_EMIT_U=8"],
    "emit_u12": ["-DVMQG_EMIT_U=12"],
    "emit_u16": ["-DVMQG_EMIT_U=16"],
    "ss_u2": ["-DVMQS_UNROLL=2"],
    "ss_kind": ["-DVMQS_KIND_SCAN=1"],
    "ss_wpe1": ["-DVMQS_WAVES_PER_EU=1"],
    "ss_wpe8_u8": ["-DVMQS_UNROLL=8"],
    "rt_tile256": ["-DVMQR_TILE_ROWS=256"],
    "rt_tile512": ["-DVMQR_TILE_ROWS=512"],
    "rt_tile512_u8": ["-DVMQR_TILE_ROWS=512", "-DVMQR_U=8"],
    "rt_tile2048": ["-DVMQR_TILE_ROWS=2048"],
    "rt_u2": ["-DVMQR_U=2"],
    "rt_u8": ["-DVMQR_U=8"],
    "nofence": ["-DVMQG_STACK_FENCES=0"],
    "emitk4_0": ["-DVMQG_EMIT_K4=0"],
    "noemitex": ["-DVMQG_EMIT_EXACT=0"],
    "emitexk2": ["-DVMQG_EMIT_EXK=2"],
    "emitexk8": ["-DVMQG_EMIT_EXK=8"],
    "emitexk1": ["-DVMQG_EMIT_EXK=1"],
    "emitexk4": ["-DVMQG_EMIT_EXK=4"],
    "ddpct67": ["-DVMQG_DD_ON_PCT=67"],
    "exact2x": ["-DVMQG_EXACT_SLOTS_PER_TOPIC=2"],
    "fxk2": ["-DVMQG_FX_K=2"],
    "fxk8": ["-DVMQG_FX_K=8"],
    "fxbpc8": ["-DVMQG_FX_BPC=8"],
    "fxk2bpc8": ["-DVMQG_FX_K=2", "-DVMQG_FX_BPC=8"],
    # the deferred look-back (r06s / r06t scripts: VMQG_AB_DIR=build/ab8, names without the fx prefix there)
    "nodefer": ["-DVMQG_FX_DEFER=0"],
    "k1bpc6": ["-DVMQG_FX_K=1", "-DVMQG_FX_BPC=6"],
    "k1bpc8": ["-DVMQG_FX_K=1", "-DVMQG_FX_BPC=8"],
    "k2bpc5": ["-DVMQG_FX_K=2", "-DVMQG_FX_BPC=5"],
    "k2bpc6": ["-DVMQG_FX_K=2", "-DVMQG_FX_BPC=6"],
    "k3": ["-DVMQG_FX_K=3"],
    "k4": ["-DVMQG_FX_K=4"],
    "bpc8": ["-DVMQG_FX_BPC=8"],
    "fxk2u2": ["-DVMQG_FX_K=2", "-DVMQG_FX_U=2"],
    "fxk2u2bpc5": ["-DVMQG_FX_K=2", "-DVMQG_FX_U=2", "-DVMQG_FX_BPC=5"],
    "fxk3": ["-DVMQG_FX_K=3"],
    "fxk6": ["-DVMQG_FX_K=6"],
    "fxpf": ["-DVMQG_FX_PREFETCH=1"],
}
OUT_DIR = os.environ.get("VMQG_AB_DIR", os.path.join(ROOT, "build", "ab"))


def build(name, flags):
    out = os.path.join(OUT_DIR, "lib_%s.so" % name)
    srcs = _lib.SOURCES
    if name.startswith("git_"):   # the library as committed at a revision (sources exported to build/ab/src_<rev>)
        rev = name[4:]
        d = os.path.join(ROOT, "build", "ab", "src_" + rev)
        os.makedirs(d, exist_ok=True)
        subprocess.run("git -C %s archive %s vernemq_amd/csrc include | tar -x -C %s" % (ROOT, rev, d), shell=True,
                       check=True)
        srcs = [os.path.join(d, "vernemq_amd", "csrc", os.path.basename(x)) for x in _lib.SOURCES]
    cmd = ["/opt/rocm/bin/hipcc"] + _lib.FLAGS + flags + ['-DVMQG_BUILD_ID="vmqg-build:%s+%s"' % (_lib.source_id(), name),
                                                          "-o", out] + srcs
    r = subprocess.run(cmd, capture_output=True, text=True)
    return name, r.returncode, r.stderr[-2000:]


if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    os.makedirs(OUT_DIR, exist_ok=True)
    with ThreadPoolExecutor(4) as ex:
        for name, rc, err in ex.map(lambda n: build(n, VARIANTS.get(n, [])), names):
            print(name, "ok" if rc == 0 else "FAILED\n" + err)
