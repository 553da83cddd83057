"""Feed-forward block ``lin_out(dropout(act(lin_in(x))))`` with the activation and dropout inside GEMM epilogues.

Reference semantics: T5 ``T5DenseActDense`` (transformers modeling_t5.py:83-94: wi -> relu -> dropout -> wo)
and BART's ``fc1 -> activation_fn -> dropout(activation_dropout) -> fc2`` (modeling_bart.py:297-301).

Through the library path (hipBLASLt + csrc/act.hip) every FFN makes two extra full passes over the
``[tokens, d_ff]`` activation — the activation+dropout kernel forward and its backward — and keeps both
the pre-activation (for the activation backward) and the activation (for the ``lin_out`` weight gradient)
alive until backward.  Here (csrc/gemm_fused.hip):

* forward:  ``H = dropout(act(X Wiᵀ + bi))`` is ONE GEMM whose epilogue applies bias, activation and the
  counter-based dropout mask (ops/rng.py, same element index as csrc/act.hip, so both paths draw identical
  masks); GELU also writes ``G = dropout'(act'(U))`` (derivative with the keep mask and scale applied) as a
  second output, so its backward epilogue is one multiply; ReLU stores nothing else;
* backward: ``dU = act'(U) · dropout'(dY Wo)`` is ONE GEMM (``dY [M, d] x Wo [d, F]``, k-major B) whose
  epilogue applies the dropout and activation backward.  For ReLU the derivative mask is ``H != 0``
  (ReLU and dropout both produce exact zeros), so the pre-activation is never stored: one
  ``[tokens, d_ff]`` tensor less per layer.  With the ping-pong kernel (variants 8 / 9, the default) the
  forward epilogue also writes that mask as bits (``M * d_ff / 32`` int32 words, 1/16 of ``H``) and the
  backward stages them through LDS instead of re-reading the bf16 ``H`` (which stays saved only as the
  ``lin_out`` weight-gradient input);
* weight gradients are accumulated straight into the flat gradient buffer (ops/gemm.py), and the
  reducer's post hooks are fired by hand exactly as ops/linear.py does.

Taken only when both linears carry FlatParams-managed gradients (``_dllm_fused_wgrad``), the input is
bf16 on the GPU and the shapes suit the kernel (tokens and d_ff multiples of 256, d_model of 64); anything
else (CPU, odd token counts) runs the unfused modules with identical semantics.  Gated FLAN-T5 FFNs take
``gated_ffn`` (one GEMM pairs gate and up columns in registers, epilogues 8 / 9).
Which kernel runs which FFN (row thresholds, GELU kernel, gated bounds) is ops/routing.py's table (``ffn*`` and
``gated_*`` keys; ``DLLM_ROUTE=ffn=unfused`` forces the unfused path for A/B runs).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext
from .activations import act_dropout
from . import gemm, routing, streams
from .gemm import bias_grad_accumulate, linear_dgrad, linear_fwd, wgrad_accumulate
from . import linear as _linear
from .linear import _fire, _fusable, _gbuf, _use

# activation -> (forward epilogue, backward epilogue) of csrc/gemm_fused.hip
EPILOGUES = {"relu": (1, 3), "gelu": (2, 4), "gelu_new": (5, 6), "gelu_fast": (5, 6)}
# kernel choices, with their evidence: ops/routing.py.  The ReLU FFN runs on csrc/gemm_w4.hip (ReLU + dropout + bit-mask
# epilogue forward, input gradient through that mask) from ``ffn_w4_min_rows`` token rows (default 0: every fused size)
# and on the ping-pong kernel below (its bit mask feeds the same w4 backward); the GELU FFN on the ping-pong kernel (``ffn_gelu`` = pp) or the w4
# GELU epilogues (= w4); FFNs under ``ffn_min_rows`` rows run unfused (hipBLASLt + the activation kernel)
w4_ffn_calls = 0
w4_gelu_calls = 0
fused_calls = 0  # number of FFN forwards that took the fused path (tests assert the kernel really ran)


def _pingpong(C, K: int) -> bool:
    """The kernel chosen for reduction length K is the ping-pong one (the only one with the ReLU bit mask)."""
    return C.gemm_fused_variant(K) in (8, 9)


def _enabled() -> bool:
    return routing.get("ffn") == "fused"


class _FusedFFNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wi, bi, wo, bo, act, p, seed, params):
        C = _ext.native()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        efwd, _ = EPILOGUES[act]
        u = mask = None
        if efwd == 1 and x2.shape[0] >= routing.get("ffn_w4_min_rows") and C.gemm_w4_supported(x2, wi, False) and \
                (bi is None or (bi.dtype == torch.bfloat16 and bi.is_contiguous())):
            global w4_ffn_calls
            w4_ffn_calls += 1
            mask = torch.empty(C.gemm_w4_mask_words(x2.shape[0], wi.shape[0]), device=x.device, dtype=torch.int32)
            h = C.gemm_w4(x2, wi, False, bi, None, False, -1, True, 1, float(p), int(seed), mask)
            y = linear_fwd(h, wo, bo)
            ctx.set_materialize_grads(False)
            ctx.save_for_backward(x2, h, None, mask)
            ctx.params = params
            for q in params:
                _use(q)
            ctx.cfg = (act, float(p), int(seed), shape)
            ctx.w4 = True
            return y.view(*shape[:-1], wo.shape[0]), x.view_as(x)
        ctx.w4 = False
        if efwd != 1:  # GELU: the backward multiplies by the stored derivative
            u = torch.empty(x2.shape[0], wi.shape[0], device=x.device, dtype=x.dtype)
        if efwd == 2 and routing.get("ffn_gelu") == "w4" and C.gemm_w4_supported(x2, wi, False) and \
                (bi is None or (bi.dtype == torch.bfloat16 and bi.is_contiguous())):
            global w4_gelu_calls
            w4_gelu_calls += 1
            h = C.gemm_w4(x2, wi, False, bi, None, False, -1, True, 11, float(p), int(seed), None, False, None, u)
            y = linear_fwd(h, wo, bo)
            ctx.set_materialize_grads(False)
            ctx.save_for_backward(x2, h, u, None)
            ctx.params = params
            for q in params:
                _use(q)
            ctx.cfg = (act, float(p), int(seed), shape)
            return y.view(*shape[:-1], wo.shape[0]), x.view_as(x)
        if efwd == 1 and _pingpong(C, x2.shape[1]) and _pingpong(C, wo.shape[0]):  # ReLU: mask bits
            mask = torch.empty(x2.shape[0] * wi.shape[0] // 32, device=x.device, dtype=torch.int32)
        h = C.gemm_fused(x2, wi, False, efwd, bi, None, u, float(p), int(seed), -1, mask)
        y = linear_fwd(h, wo, bo)
        ctx.set_materialize_grads(False)  # the residual alias's gradient is None when the caller does not use it
        ctx.save_for_backward(x2, h, u, mask)
        ctx.params = params
        for q in params:
            _use(q)
        ctx.cfg = (act, float(p), int(seed), shape)
        return y.view(*shape[:-1], wo.shape[0]), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dres):
        x2, h, u, mask = ctx.saved_tensors
        Wi, Bi, Wo, Bo = ctx.params
        act, p, seed, shape = ctx.cfg
        C = _ext.native()
        _, ebwd = EPILOGUES[act]
        wo = Wo.detach()
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not C.gemm_fused_supported(dy2, wo, True):
            dy2 = dy2.contiguous()
        # GELU: the wi bias gradient comes out of the same GEMM's epilogue as per-128-row column sums of dU
        bsum = None
        w4g = (ebwd == 4 and routing.get("ffn_gelu") == "w4" and dy2.shape[0] % 128 == 0
               and C.gemm_w4_supported(dy2, wo, True))
        if Bi is not None and ebwd in (4, 6) and (w4g or _pingpong(C, wo.shape[0])):
            bsum = torch.empty(dy2.shape[0] // 128, wo.shape[1], device=dy2.device, dtype=torch.float32)
        if w4g:  # dU = dH * (stored derivative) + per-128-row column partials, on the w4 kernel
            cs = bsum if bsum is not None else torch.empty(dy2.shape[0] // 128, wo.shape[1], device=dy2.device,
                                                           dtype=torch.float32)
            du = C.gemm_w4(dy2, wo, True, None, None, False, -1, False, 12, 0.0, 0, None, False, u, None, cs)
        elif ctx.w4:  # d-relu from the w4 forward's bit mask
            if not C.gemm_w4_supported(dy2, wo, True):
                dy2 = dy2.contiguous()
            du = C.gemm_w4(dy2, wo, True, None, None, False, -1, True, 7, p, seed, mask)
        elif mask is not None and C.gemm_w4_supported(dy2, wo, True):  # d-relu, ping-pong mask
            du = C.gemm_w4(dy2, wo, True, None, None, False, -1, True, 7, p, seed, mask, True)
        elif mask is not None:  # d-relu from the bit mask
            du = C.gemm_fused(dy2, wo, True, 7, None, None, None, p, seed, -1, mask)
        else:
            du = C.gemm_fused(dy2, wo, True, ebwd, None, h if ebwd == 3 else u, None, p, seed, -1, None, bsum)
        with torch.no_grad():
            wgrad_accumulate(_gbuf(Wo), dy2, h, async_ok=streams.site_ok(Wo))
            if Bo is not None:
                bias_grad_accumulate(_gbuf(Bo), dy2, dy, async_ok=streams.site_ok(Bo))
        _fire(Wo)
        if Bo is not None:
            _fire(Bo)
        dx = None
        if ctx.needs_input_grad[0]:  # post-LN residual (ffn_res): its gradient accumulated by this GEMM (beta = 1)
            if dres is not None and dres.is_contiguous() and dres.dtype == du.dtype and dres.shape == shape:
                # a deferred weight gradient still reads dres (ops/gemm.py WgradDefer): accumulate into a copy
                acc = dres.clone() if gemm.holds(dres) else dres
                dx = linear_dgrad(du, Wi.detach(), out=acc.view(-1, shape[-1]))
            else:
                dx = linear_dgrad(du, Wi.detach())
                if dres is not None:
                    dx = dx + dres.reshape(dx.shape)
        with torch.no_grad():
            wgrad_accumulate(_gbuf(Wi), du, x2, async_ok=streams.site_ok(Wi))
            if bsum is not None:
                gemm.colsum_partials_acc(_gbuf(Bi), bsum)  # the GELU backward GEMM's per-128-row partials
            elif Bi is not None:
                bias_grad_accumulate(_gbuf(Bi), du, async_ok=streams.site_ok(Bi))
        _fire(Wi)
        if Bi is not None:
            _fire(Bi)
        return (None if dx is None else dx.view(shape)), None, None, None, None, None, None, None, None


def _fusable_shapes(x2: torch.Tensor, wi: torch.Tensor, wo: torch.Tensor) -> bool:
    C = _ext.native()
    M, d = x2.shape
    Fd = wi.shape[0]
    return (tuple(wo.shape) == (d, Fd) and M % 256 == 0 and Fd % 256 == 0 and d % 64 == 0 and M * Fd < 2**32
            and C.gemm_fused_supported(x2, wi, False) and C.gemm_fused_supported(x2, wo, True))


class _FusedGatedFFNFn(torch.autograd.Function):
    """``wo(dropout(gelu_new(x wi_0ᵀ) * (x wi_1ᵀ)))`` with ``wi = [wi_0; wi_1]`` stacked (models/t5.py).

    Forward: ONE GEMM (csrc/gemm_fused.hip epilogue 8) pairs each gate column with its up column in registers
    and writes ``h`` plus the two backward factors ``G1 = s·gelu'(gate)·up`` and ``G2 = s·gelu(gate)``; the
    ``[tokens, 2·d_ff]`` product is never stored and there is no activation kernel.  Backward: ONE GEMM
    ``dH = dy · wo`` (epilogue 9) writes ``[dH·G1 | dH·G2]`` straight in the stacked layout that the wi
    weight gradient and dgrad consume.  Unfused: GEMM store of ``[M, 2F]`` + act kernel (read 2F, write F)
    forward, act-backward kernel (read F + 2F, write 2F) backward."""

    @staticmethod
    def forward(ctx, x, wi, wo, p, seed, params):
        C = _ext.native()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        h, g1, g2 = C.gemm_geglu(x2, wi, float(p), int(seed))
        y = linear_fwd(h, wo)
        ctx.save_for_backward(x2, h, g1, g2)
        ctx.params = params
        for q in params:
            _use(q)
        ctx.shape = shape
        return y.view(*shape[:-1], wo.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, h, g1, g2 = ctx.saved_tensors
        Wi, Wo = ctx.params
        C = _ext.native()
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not C.gemm_fused_supported(dy2, Wo.detach(), True):
            dy2 = dy2.contiguous()
        du = C.gemm_dgeglu(dy2, Wo.detach(), g1, g2)
        with torch.no_grad():
            wgrad_accumulate(_gbuf(Wo), dy2, h, async_ok=streams.site_ok(Wo))
        _fire(Wo)
        dx = linear_dgrad(du, Wi.detach()) if ctx.needs_input_grad[0] else None
        with torch.no_grad():
            wgrad_accumulate(_gbuf(Wi), du, x2, async_ok=streams.site_ok(Wi))
        _fire(Wi)
        return (None if dx is None else dx.view(ctx.shape)), None, None, None, None, None


gated_calls = 0  # number of gated FFN forwards that took the fused path
# Where the fused gated GEMMs win (ops/routing.py gated_min_mf / gated_max_d; tools/geglu_bench.py,
# profiles/r2_geglu_bench.jsonl, flan-t5 A/Bs in profiles/r2_geglu_ab.txt): they need >= 2 output tiles per CU to run
# persistent (epilogue stores / loads under the next tile's MFMAs), and with the longest reduction (d_model 2048)
# hipBLASLt's GEMM outruns the ping-pong kernel by as much as the two activation passes cost.  Since the gated
# backward's epilogue loads and stores whole rows through LDS (round 4, profiles/r4_gemm_pp_stage_ab.txt)
# flan-t5-large b=32 is 2.1 % faster fused and flan-t5-xl equal, so the bound moved from 768 to 1024.


def gated_ffn(x: torch.Tensor, lin_in, lin_out, act: str, p: float = 0.0, seed: int = 0) -> torch.Tensor:
    """``lin_out(dropout(act(x wi_0ᵀ) * (x wi_1ᵀ)))`` with ``lin_in.weight = [wi_0; wi_1]``, fused where possible
    (tanh GELU, bias-free, tokens and d_ff multiples of 256, tokens x d_ff >= ``gated_min_mf``,
    d_model <= ``gated_max_d``, ops/routing.py)."""
    global gated_calls
    wi, wo = lin_in.weight, lin_out.weight
    if (act in ("gelu_new", "gelu_fast") and _enabled() and x.dtype == torch.bfloat16 and _ext.use_native(x)
            and torch.is_grad_enabled() and lin_in.bias is None and lin_out.bias is None
            and _fusable(wi) and _fusable(wo)):
        C = _ext.native()
        x2 = x.reshape(-1, x.shape[-1])
        Fd = wo.shape[1]
        if (tuple(wi.shape) == (2 * Fd, x2.shape[1]) and tuple(wo.shape) == (x2.shape[1], Fd) and Fd % 256 == 0
                and x2.shape[0] % 256 == 0 and 2 * x2.shape[0] * Fd < 2**32
                and x2.shape[0] * Fd >= routing.get("gated_min_mf") and x2.shape[1] <= routing.get("gated_max_d")
                and C.gemm_fused_supported(x2, wi, False) and C.gemm_fused_supported(x2, wo, True)):
            gated_calls += 1
            return _FusedGatedFFNFn.apply(x, wi.detach(), wo.detach(), p, seed, (wi, wo))
    return lin_out(act_dropout(lin_in(x), act, p, seed, gated=True))


def ffn(x: torch.Tensor, lin_in, lin_out, act: str, p: float = 0.0, seed: int = 0) -> torch.Tensor:
    """``lin_out(act_dropout(lin_in(x), act, p, seed))`` (non-gated), fused where possible."""
    return ffn_res(x, lin_in, lin_out, act, p, seed, residual=False)


def ffn_res(x: torch.Tensor, lin_in, lin_out, act: str, p: float = 0.0, seed: int = 0, residual: bool = True):
    """``ffn(x)`` and, with ``residual``, ``x`` again for the caller's post-LN residual connection: on the fused path
    that residual's gradient is accumulated by the FFN's input-gradient GEMM instead of an autograd add kernel."""
    global fused_calls
    if (act in EPILOGUES and _enabled() and x.dtype == torch.bfloat16 and _ext.use_native(x)
            and torch.is_grad_enabled()
            and all(_fusable(t) for t in (lin_in.weight, lin_in.bias, lin_out.weight, lin_out.bias))):
        x2 = x.reshape(-1, x.shape[-1])
        if x2.shape[0] >= routing.get("ffn_min_rows") and _fusable_shapes(x2, lin_in.weight, lin_out.weight):
            fused_calls += 1
            bi, bo = lin_in.bias, lin_out.bias
            y, res = _FusedFFNFn.apply(x, lin_in.weight.detach(), None if bi is None else bi.detach(),
                                       lin_out.weight.detach(), None if bo is None else bo.detach(), act, p, seed,
                                       (lin_in.weight, bi, lin_out.weight, bo))
            return (y, res) if residual and _linear._RES_GEMM else (y, x) if residual else y
    y = lin_out(act_dropout(lin_in(x), act, p, seed))
    return (y, x) if residual else y
