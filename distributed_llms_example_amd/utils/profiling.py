"""Tracing / throughput instrumentation.

* ``range(name)`` / ``mark(name)``: roctx push/pop ranges and markers (``/opt/rocm/lib/libroctx64.so``
  via ctypes) around forward / backward / all-reduce / optimizer (train/engine.py) and at every gradient
  bucket launch (parallel/reducer.py; the native reducer marks through csrc/reducer.cpp), so
  ``rocprofv3 --marker-trace`` timelines are annotated; a no-op when the library is absent or
  ``DLLM_ROCTX=0``.
* ``seq2seq_train_flops``: analytic training FLOPs of one encoder-decoder step (GEMMs, attention, LM head;
  fwd + bwd = 3 x fwd), from which bench.py reports model FLOP utilisation against the MI355X dense bf16 peak.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_roctx = None
_roctx_tried = False
MI355X_BF16_DENSE_PEAK = 2.5e15


def _lib():
    global _roctx, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        if os.environ.get("DLLM_ROCTX", "1") != "0":
            for p in ("/opt/rocm/lib/libroctx64.so", "libroctx64.so"):
                try:
                    _roctx = ctypes.CDLL(p)
                    _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    _roctx.roctxMarkA.argtypes = [ctypes.c_char_p]
                    break
                except OSError:
                    continue
    return _roctx


def mark(name: str) -> None:
    """Instantaneous roctx marker (bucket launches, step boundaries)."""
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx API name
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def seq2seq_train_flops(cfg, batch: int, src: int, tgt: int) -> float:
    """Training FLOPs (fwd + bwd = 3 × fwd) of one step: dense GEMMs + attention + LM head."""
    d, f, H, dk = cfg.d_model, cfg.d_ff, cfg.num_heads, cfg.d_kv
    inner = H * dk
    ff_mult = 3 if cfg.is_gated else 2
    enc = cfg.num_layers * (2 * src * d * inner * 4 + 2 * src * d * f * ff_mult + 4 * src * src * inner)
    dec = cfg.num_decoder_layers * (2 * tgt * d * inner * 4 + 2 * tgt * d * inner * 2 + 2 * src * d * inner * 2
                                    + 2 * tgt * d * f * ff_mult + 4 * tgt * tgt * inner + 4 * tgt * src * inner)
    head = 2 * tgt * d * cfg.vocab_size
    return 3.0 * batch * (enc + dec + head)
