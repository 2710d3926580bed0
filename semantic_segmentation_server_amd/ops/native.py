"""Loading of the in-tree native modules.

``host()`` returns the host C++ module, building it on first use if the ``.so`` is
missing (g++ is always present). ``hip()`` returns the HIP kernel module; it is
built by ``__graft_entry__.build()`` / ``python -m semantic_segmentation_server_amd.ops.build``
and, when a GPU is present, its absence is an error — there is no silent eager
fallback on a GPU box (set ``SSA_ALLOW_TORCH_FALLBACK=1`` to opt into the torch
reference path explicitly).
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import threading

_lock = threading.Lock()
_mods = {}


class NativeUnavailable(RuntimeError):
    pass


def _load(name: str, builder):
    with _lock:
        if name in _mods:
            return _mods[name]
        alt = os.environ.get("SSA_HIP_SO") if name == "_hip" else None
        if alt:  # a diagnostic build of the same module (ops/build.py SSA_HIP_OUT)
            spec = importlib.util.spec_from_file_location(
                f"semantic_segmentation_server_amd.ops.{name}", os.path.abspath(alt))
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules[spec.name] = mod
            _mods[name] = mod
            return mod
        try:
            mod = importlib.import_module(f"semantic_segmentation_server_amd.ops.{name}")
        except ImportError:
            if os.environ.get("SSA_NO_AUTOBUILD"):
                raise
            builder()
            mod = importlib.import_module(f"semantic_segmentation_server_amd.ops.{name}")
        _mods[name] = mod
        return mod


def host():
    from .build import build_host
    return _load("_host", build_host)


def hip():
    from .build import build_hip
    try:
        return _load("_hip", build_hip)
    except Exception as e:  # pragma: no cover - exercised on broken installs
        raise NativeUnavailable(f"HIP extension unavailable: {e}") from e


def hip_debug():
    """The diagnostic kernels (csrc/hip_debug), built on first use."""
    from .build import build_hip_debug
    return _load("_hip_debug", build_hip_debug)


def hip_available() -> bool:
    try:
        hip()
        return True
    except NativeUnavailable:
        return False


def torch_fallback_allowed() -> bool:
    return os.environ.get("SSA_ALLOW_TORCH_FALLBACK", "0") == "1"
