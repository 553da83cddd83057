"""Linear layer whose weight gradient is accumulated by the GEMM itself into the flat gradient buffer.

With parameters living in FlatParams (parallel/flat.py) every parameter's gradient is a slice of one
gradient buffer (``p.grad`` itself, or ``p._dllm_gbuf`` when that buffer is fp32 for bf16 weights).  Through plain autograd the weight-gradient GEMM writes a fresh ``[out, in]`` tensor and
AccumulateGrad then adds it into that view — an extra read+write of every weight gradient and one
elementwise kernel per parameter per micro-batch (≈200 launches per T5-base step).  Here the backward
issues ``grad.addmm_(dyᵀ, x)`` (β = 1): hipBLASLt accumulates straight into the flat buffer in its
epilogue, and the post-accumulate hooks the gradient reducer relies on (parallel/reducer.py) are fired
by hand because AccumulateGrad never runs for the weight.

The fused path is taken only when the weight is marked by FlatParams (``_dllm_fused_wgrad``) and its
flat-buffer gradient slice is live; anything else (plain modules, ``zero_grad(set_to_none=True)``) falls back to
ordinary autograd with identical results.
"""
from __future__ import annotations


import torch
import torch.nn as nn
import torch.nn.functional as F

from . import streams
from . import gemm
from .gemm import bias_grad_accumulate, colsum_of, linear_dgrad, linear_fwd, wgrad_accumulate


def _gbuf(p: torch.Tensor | None) -> torch.Tensor | None:
    """The slice of the flat gradient buffer a fused op accumulates ``p``'s gradient into (parallel/flat.py).

    With fp32 gradients for bf16 parameters that slice cannot be ``p.grad`` (autograd insists on equal
    dtypes), so FlatParams hands it over as ``p._dllm_gbuf``; otherwise it is ``p.grad`` itself."""
    if p is None:
        return None
    g = getattr(p, "_dllm_gbuf", None)
    return g if g is not None else p.grad


def _use(p: torch.Tensor | None) -> None:
    """Forward: one more fused gradient contribution to ``p`` is pending for the coming backward.

    A parameter can feed several fused ops (the tied T5/BART embedding: encoder and decoder embedding
    lookups + the LM head); its reducer hooks must fire once, after the LAST contribution.  Forwards
    that run inside backward (activation-checkpoint recomputation) are not counted: their autograd
    nodes are never run, the original forward's are."""
    if p is None or torch._C._current_graph_task_id() != -1:
        return
    p._dllm_pending = getattr(p, "_dllm_pending", 0) + 1
    p._dllm_fused_seen = True


def _sole_writer(p: torch.Tensor) -> bool:
    """True when this op is the only one that accumulates into ``p``'s gradient in this backward (one pending fused
    contribution): its weight-gradient GEMM may then run on the side stream (ops/streams.py).  A tied weight (the
    T5 / BART embedding shared with the LM head) also receives the embedding backward's kernel on the compute stream."""
    return getattr(p, "_dllm_pending", 1) <= 1


def _fire(p: torch.Tensor) -> None:
    """Backward: one fused contribution to ``p`` has been accumulated; run the post-accumulate hooks
    (gradient reducer) when it was the last one."""
    n = getattr(p, "_dllm_pending", 1) - 1
    p._dllm_pending = n if n > 0 else 0
    if n > 0:
        return
    for h in getattr(p, "_dllm_post_hooks", ()):
        h(p)


class _LinearAccumFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, params):
        # weight/bias arrive detached (no autograd edge → no AccumulateGrad node, no double hook);
        # ``params`` carries the Parameters themselves, whose flat-buffer gradients are accumulated into below
        ctx.save_for_backward(x)
        ctx.weight, ctx.bias = params
        _use(params[0])
        _use(params[1])
        return linear_fwd(x, weight, bias)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w, bias = ctx.weight, ctx.bias
        dx = linear_dgrad(dy, w.detach()) if ctx.needs_input_grad[0] else None
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        with torch.no_grad():
            wgrad_accumulate(_gbuf(w), dy2, x2, async_ok=_sole_writer(w) and streams.site_ok(w))
            if bias is not None:
                bias_grad_accumulate(_gbuf(bias), dy2, dy, async_ok=streams.site_ok(bias))
        _fire(w)
        if bias is not None:
            _fire(bias)
        return dx, None, None, None


class _LinearResFn(torch.autograd.Function):
    """``(x Wᵀ + b, x)``: a linear layer whose input is ALSO the residual of a post-LN block (BART).

    The input's gradient is then ``d_residual + dY W``; through autograd the two halves come back from two consumers
    and are summed by a separate elementwise kernel (one [tokens, d] read-read-write per block).  Returning the
    residual as a second output of this op hands ``d_residual`` to this backward, where the input-gradient GEMM
    accumulates into it in its epilogue (``addmm_``, beta = 1): no add kernel."""

    @staticmethod
    def forward(ctx, x, weight, bias, params):
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(x)
        ctx.weight, ctx.bias = params
        _use(params[0])
        _use(params[1])
        return linear_fwd(x, weight, bias), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dres):
        (x,) = ctx.saved_tensors
        w, bias = ctx.weight, ctx.bias
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = None
        if ctx.needs_input_grad[0]:
            if dres is not None and dres.is_contiguous() and dres.dtype == dy.dtype and dres.shape == x.shape:
                # a deferred weight gradient still reads dres (ops/gemm.py WgradDefer): accumulate into a copy
                dx = linear_dgrad(dy, w.detach(), out=dres.clone() if gemm.holds(dres) else dres)
            else:
                dx = linear_dgrad(dy, w.detach())
                if dres is not None:
                    dx = dx + dres
        x2 = x.reshape(-1, x.shape[-1])
        with torch.no_grad():
            wgrad_accumulate(_gbuf(w), dy2, x2, async_ok=_sole_writer(w) and streams.site_ok(w))
            if bias is not None:
                bias_grad_accumulate(_gbuf(bias), dy2, dy, async_ok=streams.site_ok(bias))
        _fire(w)
        if bias is not None:
            _fire(bias)
        return dx, None, None, None


_RES_GEMM = True  # False: the residual gradient summed by autograd (tests flip the module attribute)


def linear_res(x: torch.Tensor, mod) -> tuple[torch.Tensor, torch.Tensor]:
    """``(mod(x), residual)`` where ``residual`` is ``x`` for the caller's residual connection; on the fused path the
    residual's gradient is accumulated by this linear's input-gradient GEMM (``_LinearResFn``)."""
    w, b = mod.weight, mod.bias
    if _RES_GEMM and torch.is_grad_enabled() and x.requires_grad and _fusable(w) and _fusable(b):
        y, res = _LinearResFn.apply(x, w.detach(), None if b is None else b.detach(), (w, b))
        _mark_bias_out(y, b is not None)
        return y, res
    return mod(x), x


def _mark_bias_out(y: torch.Tensor, on: bool) -> None:
    """Mark a biased projection's output: a consumer that sums dY over tokens on the way (ops/attention.py) hands that
    sum to the bias gradient (ops/gemm.py colsum_record).  Also on the tensor y is a full view of (the GEMM's 2-D
    result): views of y, like the attention's [B, S, 3, H, D], point at that root, not at y."""
    if not on:
        return
    y._dllm_bias_out = True
    base = y._base
    if base is not None and base.data_ptr() == y.data_ptr() and base.numel() == y.numel():
        base._dllm_bias_out = True


def _fusable(p: torch.Tensor | None) -> bool:
    return p is None or (getattr(p, "_dllm_fused_wgrad", False) and p.requires_grad and _gbuf(p) is not None)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """Functional ``F.linear`` with the weight gradient accumulated by the GEMM (e.g. a tied LM head)."""
    if torch.is_grad_enabled() and _fusable(weight) and _fusable(bias):
        y = _LinearAccumFn.apply(x, weight.detach(), None if bias is None else bias.detach(), (weight, bias))
        _mark_bias_out(y, bias is not None)
        return y
    return F.linear(x, weight, bias)


class Linear(nn.Linear):
    """Drop-in ``nn.Linear`` (same parameters / state-dict keys / init) with GEMM-fused grad accumulation."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)


# ------------------------------------------------------------------------------------------------
# One GEMM for several projections of the same input (the decoder's per-layer cross-attention K/V)


def _adjacent(ts):
    """[t0; t1; ...] as ONE view when the tensors sit back-to-back in memory (same trailing shape),
    else None.  FlatParams lays out grouped parameters this way (``_dllm_param_groups``)."""
    t0 = ts[0]
    if t0 is None or not t0.is_contiguous():
        return None
    tail = tuple(t0.shape[1:])
    rows = 0
    for t in ts:
        if (t is None or not t.is_contiguous() or tuple(t.shape[1:]) != tail or t.dtype != t0.dtype
                or t.data_ptr() != t0.data_ptr() + rows * (t0.numel() // t0.shape[0]) * t0.element_size()):
            return None
        rows += t.shape[0]
    return t0.as_strided((rows,) + tail, t0.stride())


class _StackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b, ws, bs, shape):
        y = linear_fwd(x, W, b)
        n = ws[0].shape[0]
        gbuf = torch.empty_like(y)
        outs = []
        for l in range(len(ws)):
            o = y[..., l * n:(l + 1) * n].view(shape)
            o._dllm_grad_into = gbuf[..., l * n:(l + 1) * n].view(shape)  # consumers may write dY_l here
            o._dllm_bias_out = b is not None  # ... and record its column sum there (colsum_record)
            outs.append(o)
        ctx.save_for_backward(x)
        ctx.W, ctx.gbuf, ctx.params, ctx.n = W, gbuf, (ws, bs), n
        for q in list(ws) + list(bs):
            _use(q)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        (x,) = ctx.saved_tensors
        gbuf, W, n = ctx.gbuf, ctx.W, ctx.n
        ws, bs = ctx.params
        for l, g in enumerate(grads):
            part = gbuf[..., l * n:(l + 1) * n]
            if g is None:
                part.zero_()
                continue
            mine = part.view(g.shape)
            if not (g.data_ptr() == mine.data_ptr() and g.stride() == mine.stride()):
                mine.copy_(g)  # consumer produced its own buffer
        G2 = gbuf.view(-1, gbuf.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = linear_dgrad(G2, W).view(x.shape) if ctx.needs_input_grad[0] else None
        with torch.no_grad():
            gw = _adjacent([_gbuf(w) for w in ws])
            if gw is not None:
                wgrad_accumulate(gw, G2, x2)
            else:
                dW = G2.t() @ x2
                for l, w in enumerate(ws):
                    _gbuf(w).add_(dW[l * n:(l + 1) * n])
            if bs[0] is not None:
                gb = _adjacent([_gbuf(bb) for bb in bs])
                # every layer's consumer summed its dY_l over tokens (ops/attention.py): n-column adds, no G2 pass
                cs = [colsum_of(g, n) for g in grads]
                if gb is not None and all(c is not None for c in cs):
                    gemm.colsum_handoffs += len(cs)
                    for l, c in enumerate(cs):
                        gemm.colsum_partials_acc(gb[l * n:(l + 1) * n], c)
                elif gb is not None:
                    bias_grad_accumulate(gb, G2)
                else:
                    db = G2.sum(0)
                    for l, bb in enumerate(bs):
                        _gbuf(bb).add_(db[l * n:(l + 1) * n])
        ctx.gbuf = None
        for p in list(ws) + [bb for bb in bs if bb is not None]:
            _fire(p)
        return dx, None, None, None, None, None


def stacked_linear(x, mods, shape):
    """``[mods[l](x).view(shape) for l]`` computed by ONE GEMM against the row-stacked weights.

    With the weights laid out back-to-back by FlatParams the stacked weight is a view (no copy), the
    backward is one dgrad GEMM with K = Σ n_l (instead of L GEMMs plus L-1 adds of dX) and one wgrad
    GEMM accumulated into the flat gradient buffer; consumers that know how (ops/attention.py) write
    their input gradient straight into the stacked gradient buffer through ``_dllm_grad_into``."""
    ws = [m.weight for m in mods]
    bs = [m.bias for m in mods]
    has_b = bs[0] is not None
    W = _adjacent(ws)
    B_ = _adjacent(bs) if has_b else None
    if (torch.is_grad_enabled() and W is not None and (B_ is not None or not has_b)
            and all(_fusable(w) for w in ws) and all(_fusable(b) for b in bs)):
        return list(_StackedFn.apply(x, W.detach(), None if B_ is None else B_.detach(), tuple(ws), tuple(bs), shape))
    if W is None or torch.is_grad_enabled():  # an adjacent view would route all grads to ws[0]
        W = torch.cat(ws)
    if has_b and (B_ is None or torch.is_grad_enabled()):
        B_ = torch.cat(bs)
    y = F.linear(x, W, B_)
    n = ws[0].shape[0]
    return [y[..., l * n:(l + 1) * n].view(shape) for l in range(len(mods))]
