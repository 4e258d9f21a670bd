"""vernemq_amd — MI355X-native subscription matcher behind VerneMQ's
``vmq_reg_view`` behaviour.

The product is ``libvmqgpu.so`` (HIP kernels for gfx950 + C ABI,
include/vmqg.h); this package is its host-side mirror of the reference's
view interface.  Importing it does not need a GPU; matching does.
"""
from . import _lib, subscriber, topic  # noqa: F401

__all__ = ["RegGpuView", "build"]


def build(force: bool = False) -> str:
    return _lib.build(force=force)


def __getattr__(name):
    if name == "RegGpuView":
        from .reg_view import RegGpuView
        return RegGpuView
    raise AttributeError(name)
