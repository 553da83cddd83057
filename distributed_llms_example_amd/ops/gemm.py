"""GEMM routing for the linear layers of a training step.

Who runs what (t5-base / bart-large training step, default settings):

* weight gradients ``dW (+)= dYᵀ X`` (wgrad_accumulate): csrc/gemm_w4.hip's weight-gradient mode (both operands
  token-major, K split over workgroups, fp32 split slabs summed into the flat gradient buffer by csrc/gemm.hip's
  split-K pass; round 5, 2-8 % faster than the csrc/gemm.hip kernel it replaced) from routing ``wgrad_min_rows``
  (4096) token rows; below that hipBLASLt (fp32 addmm): a 256x256-tile kernel has ~23 us of fixed cost there, 2-4x
  the library's time at the reference's batch-1 shapes (profiles/r6_wgrad_small_rows.txt);
* the FFN input GEMMs with their activation / dropout epilogues and the FFN backward through the activation
  (ops/ffn.py): csrc/gemm_fused.hip and csrc/gemm_w4.hip;
* the PLAIN projections — forward ``Y = X Wᵀ (+ b)`` of the attention q/k/v/o and FFN output layers, and the LM
  head — go to the library (hipBLASLt through torch, with the TunableOp table in configs/tunableop/): csrc/gemm_w4.hip
  ties it on these shapes in isolation and lost 0.8 % of the step in situ (profiles/r3_w4_routing_ab.txt).  Their input
  gradients ``dX (+)= dY W`` run on csrc/gemm_w4.hip from 16K token rows at any layer width (its early-release schedule
  beats the library on every such shape, profiles/r6_w4_early_release_ab.txt), on hipBLASLt below.  The choice is
  ops/routing.py's table (``proj_fwd`` / ``proj_dgrad``).

Weight-gradient GEMM notes:

Both operands are token-major ([tokens, features]), the reduction runs over tokens (10⁴-10⁵), and the
result is accumulated straight into the flat gradient buffer (bf16, or fp32 for fp32 gradient
accumulation).  Shapes the kernel does not cover (N not a multiple of 256, M not of 8, token counts not
multiples of 64, CPU tensors) go to
``torch.addmm`` (hipBLASLt / CPU BLAS).
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn.functional as F

from .. import _ext
from . import routing, streams

# Routing of the projection GEMMs: ops/routing.py ("proj_fwd", "proj_dgrad" and its row threshold; the evidence is cited
# there).
w4_calls = 0  # projections that ran on csrc/gemm_w4.hip (tests assert the kernel really ran)
colsum_handoffs = 0  # bias gradients taken from a norm backward's column sums (bias_grad_accumulate)


def _w4_ok(a: torch.Tensor, b: torch.Tensor, kmajor: bool) -> bool:
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not _ext.use_native(a):
        return False
    if kmajor:  # input gradients
        mode = routing.get("proj_dgrad")
        if mode == "lib":
            return False
        if mode == "rows" and a.shape[0] < routing.get("proj_dgrad_min_rows"):
            return False
    else:  # forwards: all on w4, none, or (narrow) the K <= 1024, N <= 4096 projections of >= proj_fwd_min_rows tokens
        mode = routing.get("proj_fwd")
        if mode == "lib":
            return False
        if mode == "narrow" and (a.shape[0] < routing.get("proj_fwd_min_rows") or a.shape[1] > 1024
                                 or b.shape[0] > 4096):
            return False
    return bool(_ext.native().gemm_w4_supported(a, b, kmajor))


def linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """``x @ wᵀ (+ bias)`` for x ``[..., K]``, w ``[N, K]`` (nn.Linear layout)."""
    global w4_calls
    x2 = x.reshape(-1, x.shape[-1])
    if _w4_ok(x2, w, False) and (bias is None or (bias.dtype == torch.bfloat16 and bias.is_contiguous())):
        w4_calls += 1
        return _ext.native().gemm_w4(x2, w, False, bias).view(*x.shape[:-1], w.shape[0])
    return F.linear(x, w, bias)


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Input gradient ``dy @ w`` for dy ``[..., N]``, w ``[N, K]``; with ``out`` (``[..., K]``, contiguous) the product
    is accumulated into it in the GEMM epilogue (``out += dy @ w``, the post-LN residual's gradient)."""
    global w4_calls
    dy2 = dy.reshape(-1, dy.shape[-1])
    if _w4_ok(dy2, w, True):
        w4_calls += 1
        if out is not None:
            _ext.native().gemm_w4(dy2, w, True, None, out.view(-1, out.shape[-1]), True)
            return out
        return _ext.native().gemm_w4(dy2, w, True).view(*dy.shape[:-1], w.shape[1])
    if out is not None:
        out.view(-1, out.shape[-1]).addmm_(dy2, w)
        return out
    return torch.matmul(dy, w)

def _native_ok(dy2: torch.Tensor, x2: torch.Tensor, out: torch.Tensor) -> bool:
    if not _ext.use_native(dy2):
        return False
    return bool(_ext.native().gemm_wgrad_supported(dy2, x2, out))


class WgradDefer:
    """Weight gradients of a gradient-accumulation window deferred to its last micro-batch.

    With small micro-batches (the reference's train-torchrun default is batch 1 x GA 16, ref/train-torchrun.py:119,126)
    each weight-gradient GEMM reduces over a few thousand tokens: split over all CUs for occupancy, its fp32 split
    slabs and their reduction cost as much as the product (profiles/r5_t5base_b8_ga16_summary.txt: wgrad + split-K
    pass 31 % of the step).  Deferred, every no_sync micro-batch only keeps its (dY, X) operand pairs alive and the
    last micro-batch runs ONE GEMM per weight over the concatenated tokens of the whole window — the same sum, at the
    efficiency of a large batch.  Readiness for the gradient reducer is unchanged: a weight's gradient is complete in
    the last micro-batch's backward, where its hook fires (bucket overlap as before).  The kept operands cost what the
    activations of one coalesced batch would; ``mem_cap`` bytes allocated ends a window's deferral early (flush)."""

    def __init__(self, mem_cap: int | None = None):
        self.segs: dict = {}  # (ptr, shape, stride, dtype) of the gradient view -> [out, beta, [(dy2, x2, v), ...]]
        self.held: set = set()  # storages of kept dY operands: nothing may write into them (holds())
        # per-block column partials of norm weight / bias gradients (ops/norms.py): reduced once per window
        self.psegs: dict = {}  # key of the gradient view -> [out, [part [G, d], ...]]
        self.final = False
        self.active = True
        self.mem_cap = mem_cap
        self.deferred = 0  # operand pairs kept (tests)
        self.merged = 0    # GEMMs that ran over a concatenated window

    @staticmethod
    def key(out):
        return (out.data_ptr(), tuple(out.shape), tuple(out.stride()), out.dtype)

    @staticmethod
    def run(out, parts, beta):
        """``out (+)= Σ dY_iᵀ X_i`` over the window: the w4 weight-gradient kernel reading every kept segment in place
        (csrc/bind.cpp gemm_wgrad_segs; equal-shaped segments, 32 per launch), else one GEMM over the concatenated
        operands.  A kept dY changed in place since it was kept (its version moved) fails loudly."""
        for dy2, _, v in parts:
            if dy2._version != v:
                raise RuntimeError("deferred weight-gradient operand modified in place (a writer must check holds())")
        dys, xs = [p[0] for p in parts], [p[1] for p in parts]
        d0, x0 = dys[0], xs[0]
        if (d0.shape[0] * len(dys) >= routing.get("wgrad_min_rows") and _native_ok(d0, x0, out)
                and all(d.shape == d0.shape and d.stride() == d0.stride() for d in dys)
                and all(x.shape == x0.shape and x.stride() == x0.stride() for x in xs)):
            C = _ext.native()
            for g in range(0, len(dys), 32):
                C.gemm_wgrad_segs(dys[g:g + 32], xs[g:g + 32], out, beta or g > 0)
            return out
        return _wgrad(out, torch.cat(dys), torch.cat(xs), beta)

    def pending(self) -> bool:
        """Kept weight-gradient operands or norm partials that no GEMM / reduction has consumed yet."""
        return bool(self.segs or self.psegs)

    @torch.no_grad()
    def flush(self) -> None:
        """Every pending window now (compute stream): the end of the last micro-batch's backward, or the memory cap."""
        segs, self.segs = self.segs, {}
        psegs, self.psegs = self.psegs, {}
        self.held = set()
        for out, beta, parts in segs.values():
            self.merged += 1
            self.run(out, parts, beta)
        for out, parts in psegs.values():
            self.merged += 1
            colsum_partials_acc(out, torch.cat(parts) if len(parts) > 1 else parts[0])

    def partials(self, out: torch.Tensor, part: torch.Tensor | None = None) -> list | None:
        """A norm backward's per-block partials of ``out``'s gradient: kept (no_sync micro-batch; returns None), or —
        in the window's last micro-batch — the kept ones for the caller to reduce with its own (returns the list)."""
        k = self.key(out)
        if not self.final:
            self.psegs.setdefault(k, [out, []])[1].append(part)
            self.deferred += 1
            return None
        ent = self.psegs.pop(k, None)
        return ent[1] if ent is not None else []


_defer: list = [None]


def deferring() -> WgradDefer | None:
    """The active deferral window (:func:`defer_wgrads`), if any."""
    return _defer[0]


def holds(t: torch.Tensor | None) -> bool:
    """``t`` shares storage with a kept (deferred) dY operand: a caller about to write into t in place (a dgrad GEMM
    accumulating into the residual gradient, ops/linear.py / ops/ffn.py) must write elsewhere instead."""
    d = _defer[0]
    return bool(t is not None and d is not None and d.held and t.untyped_storage().data_ptr() in d.held)


@contextlib.contextmanager
def defer_wgrads(d: WgradDefer | None, final: bool):
    """Weight gradients inside go to ``d`` (no_sync micro-batches: kept; ``final``: merged with what was kept)."""
    prev = _defer[0]
    _defer[0] = d if d is not None and d.active else None
    if d is not None:
        d.final = final
    try:
        yield
    finally:
        _defer[0] = prev


@torch.no_grad()
def wgrad_accumulate(out: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, beta: bool = True,
                     async_ok: bool = True, defer: bool = True) -> torch.Tensor:
    """``out (+)= dy2ᵀ @ x2`` with dy2 = [T, M], x2 = [T, N], out = [M, N].  Inside an ops/streams.py scope (and with
    ``async_ok``: no compute-stream kernel accumulates into ``out`` in the same backward) it runs on the side stream.
    Inside :func:`defer_wgrads` the product joins the window's deferred GEMM (:class:`WgradDefer`) — unless ``defer``
    is False: the caller reuses dy2's memory afterwards (the LM head's vocabulary-chunk scratch)."""
    d = _defer[0] if defer else None
    if d is not None:
        k = WgradDefer.key(out)
        ent = d.segs.pop(k, None) if (d.final or not beta) else d.segs.get(k)
        if not beta:
            ent = None  # overwritten: what was kept no longer counts
        if not d.final:
            if ent is None:
                d.segs[k] = ent = [out, beta, []]
            ent[2].append((dy2, x2, dy2._version))
            d.held.add(dy2.untyped_storage().data_ptr())
            d.deferred += 1
            return out
        if ent is not None:
            parts = ent[2] + [(dy2, x2, dy2._version)]
            beta = ent[1]
            d.merged += 1
            fn = lambda: WgradDefer.run(out, parts, beta)  # noqa: E731
            if async_ok:
                return streams.run(fn, *[t for p in parts for t in p[:2]])
            return fn()
    if async_ok:
        return streams.run(lambda: _wgrad(out, dy2, x2, beta), dy2, x2)
    return _wgrad(out, dy2, x2, beta)


def _wgrad(out, dy2, x2, beta):
    if dy2.shape[0] >= routing.get("wgrad_min_rows") and _native_ok(dy2, x2, out):
        _ext.native().gemm_wgrad(dy2, x2, out, beta, -1, 0)
        return out
    if out.dtype != dy2.dtype:  # fp32 gradient buffer, bf16 operands: the product itself in fp32, then one fp32 add
        if dy2.is_cuda and beta:  # accumulated in the GEMM (fp32 C, bf16 operands)
            return torch.addmm(out, dy2.t(), x2, out_dtype=out.dtype, out=out)
        if dy2.is_cuda:
            g = torch.mm(dy2.t(), x2, out_dtype=out.dtype)  # fp32 output from bf16 operands (no bf16 rounding)
        else:
            g = torch.mm(dy2.t().to(out.dtype), x2.to(out.dtype))
        return out.add_(g) if beta else out.copy_(g)
    if beta:
        return out.addmm_(dy2.t(), x2)
    return torch.mm(dy2.t(), x2, out=out)


@torch.no_grad()
def bias_grad_accumulate(out: torch.Tensor, dy2: torch.Tensor, dy: torch.Tensor | None = None,
                         async_ok: bool = True) -> torch.Tensor:
    """``out += dy2.sum(0)`` (bias gradient of a linear layer, accumulated in place).  ``dy``: the gradient tensor as
    autograd delivered it; when its producer already summed it over tokens (:func:`colsum_record`: the BART post-LN
    backward kernel, the attention backward kernels) that fp32 column sum is added instead of re-reading dy."""
    global colsum_handoffs
    cs = colsum_of(dy, out.numel())
    if cs is not None:
        colsum_handoffs += 1
        if not async_ok:
            return colsum_partials_acc(out, cs)
        return streams.run(lambda: colsum_partials_acc(out, cs), cs)
    if not async_ok:
        return _colsum(out, dy2)
    return streams.run(lambda: _colsum(out, dy2), dy2)


def colsum_record(t: torch.Tensor, cs: torch.Tensor) -> None:
    """Attach ``cs`` = fp32 partial column sums [G, n] of ``t.reshape(-1, n)`` (rows summing to its column sum),
    computed by t's producer on the way (the BART post-LN backward kernel, ops/norms.py; the attention backward kernels'
    dQ / dK / dV epilogues, ops/attention.py), for the bias gradient of the linear layer that consumes t's gradient
    (:func:`bias_grad_accumulate`: one reduce-and-accumulate kernel)."""
    t._dllm_colsum = (cs, t._version, t.numel(), t.data_ptr())


def colsum_partials_acc(out: torch.Tensor, part: torch.Tensor) -> torch.Tensor:
    """``out += part.sum(0)`` (fp32 partials [G, n] into an fp32 / bf16 [n] gradient): csrc/norm.hip's column
    reduction straight into the flat gradient buffer."""
    part = part.reshape(-1, out.numel())
    if part.is_cuda and out.is_contiguous() and part.is_contiguous() and out.dtype in (torch.float32, torch.bfloat16):
        _ext.native().colsum_partials_acc(part, out.view(-1))
        return out
    return out.add_(part.sum(0).view_as(out).to(out.dtype))


def colsum_of(dy: torch.Tensor | None, n: int) -> torch.Tensor | None:
    """The column sum recorded on ``dy`` — or on its base, when autograd delivers a full view of the producer's tensor
    (the [B, S, 3, H, D] attention gradient as the projection's [B, S, 3 d]) — if it still describes dy: same storage,
    element count and version (an in-place accumulation of another consumer's gradient bumps the version and the sum
    no longer describes dy); ``n`` = the bias length.  None otherwise."""
    if dy is None:
        return None
    rec = getattr(dy, "_dllm_colsum", None)
    if rec is None and dy._base is not None:
        rec = getattr(dy._base, "_dllm_colsum", None)
    if rec is None:
        return None
    cs, ver, numel, ptr = rec
    if cs.shape[-1] == n and dy._version == ver and dy.numel() == numel and dy.data_ptr() == ptr:
        return cs
    return None


def _colsum(out, dy2):
    if _ext.use_native(dy2) and dy2.dtype == torch.bfloat16 and dy2.stride(-1) == 1 and dy2.shape[-1] % 2 == 0 \
            and dy2.stride(0) % 2 == 0 and out.is_contiguous():
        _ext.native().colsum_acc(dy2, out)
        return out
    return out.add_(dy2.sum(0).to(out.dtype))
