"""Weight-gradient GEMMs on a side HIP stream, overlapping the input-gradient chain of the backward pass.

In backward every linear layer issues two independent GEMMs: the input gradient ``dX = dY W`` (the next layer's
backward waits for it) and the weight gradient ``dW += dYᵀ X`` (nothing in the backward waits for it).  On one stream
they serialise, and at the reference's small micro-batches (1-8 samples per GPU: a [1024 x 768] x [768 x 2304] GEMM is
36 of the 256 CUs' worth of 256x256 tiles) each kernel leaves most of the chip idle.  Here the weight gradient (and the
bias gradient) is launched on a side stream that forks from the compute stream at that point, so the chip runs it
beside the following input-gradient / attention-backward kernels.

Ordering and memory, without ``record_stream``:

* fork: the side stream waits on the compute stream before each launch (dY, X and the gradient buffer are ready);
* lag: after each launch the compute stream waits on the side work launched ``LAG`` launches earlier and only then
  drops this module's references to that work's inputs, so the caching allocator never reuses a block the side
  stream may still read, and at most ``LAG`` layers' inputs are held beyond their autograd lifetime;
* join: the end of the backward (``scope`` exit, engine.forward_backward) joins the side stream into the compute stream,
  before the gradient all-reduce and the optimizer read the gradients.

All three are stream waits, so a HIP-graph capture records them as graph edges (train/graph.py).

Paired mode (``DLLM_ROUTE=wgrad_stream_sites=qkv+wi+...``, the layer roles of the parameters: the name of the module that
owns the weight, e.g. T5 ``qkv`` / ``o`` / ``wi`` / ``wo``, BART ``qkv_proj`` / ``out_proj`` / ``fc1`` / ``fc2``): only
those layers' weight gradients go to the side stream, at any micro-batch size, and instead of the lagged joins the
compute stream joins at the end of the NEXT memory- or VALU-bound backward op (``pair_join``: the norm backward,
the attention backward) — so a weight-gradient GEMM (MFMA-bound) runs beside a kernel that leaves the matrix cores
idle, never beside another GEMM (the all-sites mode's loss at large batch).  Not used when a
gradient reducer launches bucket all-reduces from the autograd hooks during the backward (those order themselves
after the compute stream only), nor for gradients another compute-stream kernel also accumulates into (the tied
embedding's LM-head slice: ops/lm_head.py keeps those synchronous).  Used for small micro-batches only
(``default_enabled``).
"""
from __future__ import annotations

import collections
import contextlib
import re

import torch

from . import routing

LAG = max(1, int(routing.get("wgrad_stream_lag")))
_SITES_RAW = str(routing.get("wgrad_stream_sites"))
SITES = frozenset(s for s in re.split(r"[,+]", _SITES_RAW) if s) if _SITES_RAW else None
_on = [False]
_side: dict = {}
_used: set = set()  # devices whose side stream has work since the last join
_pending: collections.deque = collections.deque()
launches = 0  # side-stream launches since import (tests assert the path really ran)


def default_enabled(tokens: int | None = None) -> bool:
    """ops/routing.py ``wgrad_stream``: ``auto`` (default) = on for micro-batches of at most
    ``wgrad_stream_max_tokens`` input tokens (default 32768), where single kernels leave the chip partly idle; off
    above, where two full-chip GEMMs side by side only compete (t5-base, one MI355X, interleaved: batch 1 +9.8 %,
    batch 8 x GA 16 +4.2 %, batch 512 -3.6 %, profiles/r4_wgrad_stream_ab.txt); ``1`` always; ``0`` never."""
    mode = str(routing.get("wgrad_stream"))
    if mode == "0":
        return False
    if SITES is not None:
        return bool(SITES)
    if mode == "1" or tokens is None:
        return True
    return tokens <= int(routing.get("wgrad_stream_max_tokens"))


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    s = _side.get(dev)
    if s is None:
        s = _side[dev] = torch.cuda.Stream(dev)
    return s


def site_ok(p) -> bool:
    """May the weight gradient of parameter ``p`` go to the side stream?  All of them, unless paired mode names the
    layer roles (``_dllm_role``: tools set it from the parameter names, train/engine.py tag_roles)."""
    return SITES is None or getattr(p, "_dllm_role", None) in SITES


def pair_join() -> None:
    """Paired mode: the end of a backward op that side-stream weight gradients were paired with."""
    if SITES is not None and _used:
        join()


def tag_roles(module: torch.nn.Module) -> None:
    """``_dllm_role`` of every weight / bias: the name of the module owning it (``qkv``, ``wi``, ``fc1`` ...)."""
    for name, p in module.named_parameters():
        parts = name.split(".")
        if len(parts) >= 2:
            p._dllm_role = parts[-2]


def run(fn, *refs):
    """``fn()`` on the side stream when a scope is active and the tensors are on the GPU, else inline.  ``refs``: the
    tensors ``fn`` reads (kept alive until the compute stream has waited for ``fn``)."""
    global launches
    if not _on[0] or not refs or not refs[0].is_cuda:
        return fn()
    dev = refs[0].device
    cur = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    side.wait_stream(cur)
    _used.add(dev)
    with torch.cuda.stream(side):
        r = fn()
    ev = torch.cuda.Event()
    ev.record(side)
    _pending.append((ev, refs, dev))
    launches += 1
    while SITES is None and len(_pending) > LAG:
        e, _, d = _pending.popleft()
        torch.cuda.current_stream(d).wait_event(e)
    return r


def join() -> None:
    """Compute stream waits for every side-stream launch since the last join; their inputs may be released.  Only
    streams with new work are joined: in a graph capture, a wait on a side stream that never forked from the capture
    stream would be a dependency on work outside the graph."""
    for dev in _used:
        torch.cuda.current_stream(dev).wait_stream(_side[dev])
    _used.clear()
    _pending.clear()


@contextlib.contextmanager
def scope(enabled: bool = True):
    """Weight gradients of the backward run inside go to the side stream; joined on exit."""
    prev = _on[0]
    _on[0] = bool(enabled) and torch.cuda.is_available()
    try:
        yield
    finally:
        _on[0] = prev
        if not prev:
            join()
