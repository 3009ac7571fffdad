"""kbgpu — MI355X-native allocate path of kube-batch v0.4 (scostache/kube-arbitrator).

Host mirror of the reference's framework/plugin surface over the C ABI in
include/kbgpu.h (libkbgpu.so: HIP kernels for gfx950 + C++ ordering engine).
"""
from . import _abi, actions, api, cache, conf, framework  # noqa: F401
from ._abi import KbgError  # noqa: F401

__all__ = ["api", "cache", "conf", "framework", "actions", "KbgError"]
