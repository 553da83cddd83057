"""Loader for the in-tree native extension ``_C`` (HIP kernels + C++ runtime, built for gfx950).

Policy (round-end driver records which .so files the GPU tests load): on a GPU tensor every op
dispatches to the HIP kernel library; if the extension is missing on a GPU box the op raises
instead of silently falling back to eager PyTorch.  ``DLLM_REFERENCE_OPS=1`` forces the pure-torch
reference implementations (used as numerics oracles in tests and on CPU).
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys

import torch

_C = None
_err: Exception | None = None
_PKG = os.path.dirname(os.path.abspath(__file__))
_CSRC = os.path.join(os.path.dirname(_PKG), "csrc")


def stale_sources() -> list[str]:
    """Native sources whose content differs from what the in-tree library was built from (tools/build_native.py
    provenance record ``_C.build.json``); empty when they match or when there is no record / source tree to check."""
    import glob
    import hashlib
    import json
    rec_path = os.path.join(_PKG, "_C.build.json")
    if not (os.path.exists(rec_path) and os.path.isdir(_CSRC)):
        return []
    with open(rec_path) as f:
        built = json.load(f).get("sources", {})
    cur = {}
    for p in glob.glob(os.path.join(_CSRC, "*.hip")) + glob.glob(os.path.join(_CSRC, "*.cpp")) + \
            glob.glob(os.path.join(_CSRC, "*.h")):
        with open(p, "rb") as f:
            cur[os.path.basename(p)] = hashlib.sha256(f.read()).hexdigest()
    return sorted(k for k in set(built) | set(cur) if built.get(k) != cur.get(k))


def _load():
    global _C, _err
    if _C is not None or _err is not None:
        return _C
    try:
        path = os.environ.get("DLLM_NATIVE_SO")  # an alternative build of _C (tools/asan_host.py: host ASAN/UBSan)
        if path:
            spec = importlib.util.spec_from_file_location("distributed_llms_example_amd._C", path)
            _C = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_C)
            sys.modules["distributed_llms_example_amd._C"] = _C
        else:
            stale = stale_sources()
            if stale:  # a library built from other sources than the tree's: never run it silently
                raise ImportError(f"the in-tree _C was built from different sources ({', '.join(stale)}); rebuild "
                                  "with `python tools/build_native.py`")
            _C = importlib.import_module("distributed_llms_example_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _C = None
        _err = e
    return _C


def native():
    """The extension module, or None if it is not built."""
    return _load()


def load_error():
    _load()
    return _err


def force_reference() -> bool:
    return os.environ.get("DLLM_REFERENCE_OPS", "0") == "1"


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on the GPU and the HIP path must run."""
    if not t.is_cuda or force_reference():
        return False
    if _load() is None:
        raise RuntimeError(
            "distributed_llms_example_amd._C (HIP kernels for gfx950) is not built/loadable: "
            f"{_err!r}. Build it with `python tools/build_native.py` (or __graft_entry__.build()).")
    return True
