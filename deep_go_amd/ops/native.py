"""Loading of the in-tree native extensions.

``hip()`` returns the ``_dghip`` module (CDNA4 kernels).  On a machine with a GPU a
missing or stale extension is a hard error — there is deliberately no silent PyTorch
fallback for the GPU compute path.  ``cpu()`` returns ``_dgcpu`` (Go engine, t7 codec,
SGF parser, loader thread pool).  Both are built by ``python -m deep_go_amd._build``
(also run by ``__graft_entry__.build()``); set ``DG_AUTOBUILD=1`` to build on first use.
"""
from __future__ import annotations

import importlib
import os
import sys
from pathlib import Path

import torch  # noqa: F401  (must be loaded first: it provides libamdhip64.so.7 / librccl.so.1)

_NATIVE_DIR = Path(__file__).resolve().parent.parent / "_native"
_mods = {}


class NativeExtensionMissing(RuntimeError):
    pass


def _load(name: str):
    if name in _mods:
        return _mods[name]
    if str(_NATIVE_DIR) not in sys.path:
        sys.path.insert(0, str(_NATIVE_DIR))
    try:
        mod = importlib.import_module(name)
    except ImportError as e:
        if os.environ.get("DG_AUTOBUILD", "0") == "1":
            from .. import _build
            {"_dghip": _build.build_hip, "_dgcomm": _build.build_comm}.get(
                name, _build.build_cpu)()
            mod = importlib.import_module(name)
        else:
            raise NativeExtensionMissing(
                f"native extension {name} not built ({e}); run `python -m deep_go_amd._build`"
            ) from e
    _mods[name] = mod
    return mod


def hip():
    return _load("_dghip")


def cpu():
    return _load("_dgcpu")


def comm():
    """_dgcomm: native RCCL communicator (csrc/comm/comm.cpp)."""
    return _load("_dgcomm")


def hip_available() -> bool:
    try:
        hip()
        return True
    except NativeExtensionMissing:
        return False


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)
