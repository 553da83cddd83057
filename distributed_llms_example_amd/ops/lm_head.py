"""LM head + (label-smoothed) cross-entropy over vocabulary chunks: the ``[tokens, V]`` logits never exist.

Reference path: ``model(**batch).loss`` (ref/train-accelerator.py:220-221, ref/train-task.py:289-290) computes
``lm_head(decoder_output)`` → ``[B·T, V]`` logits → ``CrossEntropyLoss`` (T5: ``d_model^-0.5`` on the decoder
output, modeling_t5.py:1044-1045; BART: ``+ final_logits_bias``, modeling_bart.py:940; the Trainer's label
smoother for ``label_smoothing_factor``).  Materialised in bf16 that is ``B·T·V·2`` bytes (1.05 GB at t5-base,
b=128; 3.3 GB for BART-large b=32 at 1024 target tokens), written by the GEMM, read by the CE forward, read +
written by its backward, read twice more by the input- and weight-gradient GEMMs.

Here the vocabulary is processed in chunks of ``Vc`` columns sized so a chunk of logits (``N·Vc·2`` bytes,
≤ ops/routing.py ``lmhead_chunk_mb``, default 128 MiB) stays resident in the MI355X's 256 MiB Infinity Cache:

* forward: per chunk one GEMM ``h·W_cᵀ`` into a reused buffer, then csrc/ce.hip ``ce_chunk_fwd`` merges the
  chunk into a per-row online state {max, Σexp, Σx, x_label}; the last chunk writes loss_row and lse;
* backward: per chunk the logits GEMM again, ``ce_chunk_bwd`` turns them into ``g·(softmax - target)`` in place,
  then the input-gradient GEMM (accumulated in fp32) and the weight-gradient GEMM straight into the weight's
  slice of the flat gradient buffer (ops/gemm.py, ragged-M wgrad kernel), reducer hooks fired once at the end.

The price is one extra logits GEMM per step (the recompute); the gain is memory (no ``[N, V]`` tensor, no
``[N, V]`` gradient) and cache-resident CE passes.  Used when the full logits would exceed
``lmhead_full_mb`` (default 16384 MiB — sized for the 288 GB HBM: the t5-base bench at 512 samples per GPU keeps
its 4 GiB of logits and runs 1.7 % faster than chunked, ``profiles/r3_lmhead_b512_ab.txt``; ``0`` = always chunked,
``-1`` = never), or explicitly by callers.

GEMM-fused variant (``_LMHeadCEFusedFn``, the no-materialised-logits path unless ``lmhead`` = logits; see
``use_fused``): the cross-entropy runs INSIDE the logits GEMM's epilogue (csrc/gemm_w4.hip W4_EPI_CEF / W4_EPI_CEB):

* forward: ONE GEMM over the whole vocabulary whose epilogue reduces every row's 128-column half tile to an
  online-softmax partial {max, Σexp, Σx} (+ the label's logit) straight from the fp32 accumulators — the logits are
  never written, not even in bf16 — and csrc/ce.hip ``ce_merge`` folds the ``[N, V/128]`` partials into loss and lse;
* backward: per vocabulary chunk the GEMM recomputes the logits and its epilogue writes ``g·(softmax - target)`` as
  bf16 dlogits directly (no logits round trip, no separate CE pass), then the input- and weight-gradient GEMMs.
"""
from __future__ import annotations


import torch
import torch.nn.functional as F

from .. import _ext
from . import gemm as _gemm
from . import routing
from .gemm import wgrad_accumulate
from .linear import _fire, _fusable, _gbuf, _use


def _chunk_cols(N: int, V: int) -> int:
    mb = float(routing.get("lmhead_chunk_mb"))
    c = int(mb * 2**20 / (2 * max(N, 1))) // 256 * 256
    c = max(256, min(c, (V + 255) // 256 * 256))
    if V % 8 and c >= V:  # a ragged vocabulary needs >= 2 chunks (the tail chunk re-covers aligned columns)
        c = max(8, (V // 2 + 255) // 256 * 256)
    return c


def _chunks(V: int, vc: int):
    """(first column, width, leading columns to skip) per chunk.  Widths are multiples of 8 (the CE kernels' 4-wide
    vectors, 16-B aligned logits rows): a ragged vocabulary tail (BART: 50265) re-covers the last few columns of the
    previous chunk and skips them."""
    out = []
    for c0 in range(0, V, vc):
        n = min(vc, V - c0)
        if n % 8 and V >= 8:
            n8 = min(V, (n + 7) // 8 * 8)
            out.append((V - n8, n8, n8 - n))
        else:
            out.append((c0, n, 0))
    return out


def use_chunked(N: int, V: int) -> bool:
    lim = float(routing.get("lmhead_full_mb"))
    if lim < 0:
        return False
    return N * V * 2 > lim * 2**20


def wants_lm_head_loss(hidden: torch.Tensor, N: int, V: int) -> bool:
    """Whether a model's training loss goes through :func:`lm_head_loss` (no materialised logits): when the full
    logits would exceed ``lmhead_full_mb`` (use_chunked), or always with ``lmhead`` = fused (bf16 GPU)."""
    if use_chunked(N, V):
        return True
    return (routing.get("lmhead") == "fused" and hidden.dtype == torch.bfloat16
            and hidden.shape[-1] % 64 == 0 and _ext.use_native(hidden))


def _reference(h, w, labels, bias, smoothing, ignore_index):
    logits = F.linear(h.float(), w.float())
    if bias is not None:
        logits = logits + bias.float()
    return F.cross_entropy(logits, labels, ignore_index=ignore_index, label_smoothing=smoothing)


def _logits(h: torch.Tensor, wc: torch.Tensor, out: torch.Tensor) -> None:
    """One chunk of logits ``h @ wcᵀ`` into ``out`` (csrc/gemm_w4.hip when the shape allows, else hipBLASLt)."""
    if _gemm._w4_ok(h, wc, False):  # out: a fresh contiguous [N, n] view, n % 8 == 0
        _gemm.w4_calls += 1
        _ext.native().gemm_w4(h, wc, False, None, out)
    else:
        torch.mm(h, wc.t(), out=out)


def _dh_accumulate(dh: torch.Tensor, g: torch.Tensor, wc: torch.Tensor) -> None:
    """``dh += g @ wc`` with the fp32 accumulator ``dh`` read and written by the GEMM itself (beta = 1): no bf16
    product, no separate add pass over ``[N, d]`` per chunk."""
    if dh.is_cuda:
        torch.addmm(dh, g, wc, out_dtype=torch.float32, out=dh)
    else:
        dh += torch.mm(g.float(), wc.float())


class _LMHeadCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w, bias, labels, smoothing, ignore_index, params):
        C = _ext.native()
        N, d = h.shape
        V = w.shape[0]
        vc = _chunk_cols(N, V)
        buf = torch.empty(N * min(vc + 8, V), dtype=h.dtype, device=h.device)
        state = torch.empty(N, 4, dtype=torch.float32, device=h.device)
        loss_rows = torch.empty(N, dtype=torch.float32, device=h.device)
        lse = torch.empty(N, dtype=torch.float32, device=h.device)
        bias32 = bias.float().contiguous() if bias is not None else None
        chunks = _chunks(V, vc)
        for j, (c0, n, skip) in enumerate(chunks):
            lg = buf[:N * n].view(N, n)
            _logits(h, w[c0:c0 + n], lg)
            C.ce_chunk_fwd(lg, labels, bias32, state, loss_rows, lse, c0, V, float(smoothing), int(ignore_index),
                           j == 0, j + 1 == len(chunks), skip)
        count = (labels != ignore_index).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(h, w, labels, lse, count)
        ctx.bias32 = bias32
        ctx.cfg = (float(smoothing), int(ignore_index), vc)
        ctx.params = params
        if params is not None:
            _use(params[0])
        return loss_rows.sum() / count

    @staticmethod
    def backward(ctx, g):
        C = _ext.native()
        h, w, labels, lse, count = ctx.saved_tensors
        smoothing, ignore_index, vc = ctx.cfg
        N, d = h.shape
        V = w.shape[0]
        scale = (g.float() / count).reshape(1)
        p = ctx.params[0] if ctx.params is not None else None
        gw = _gbuf(p) if p is not None else None
        dw = torch.zeros_like(w, dtype=torch.float32) if (gw is None and ctx.needs_input_grad[1]) else None
        dh = torch.zeros(N, d, dtype=torch.float32, device=h.device)
        buf = torch.empty(N * min(vc + 8, V), dtype=h.dtype, device=h.device)
        for c0, n, skip in _chunks(V, vc):
            lg = buf[:N * n].view(N, n)
            wc = w[c0:c0 + n]
            _logits(h, wc, lg)
            C.ce_chunk_bwd(scale, lg, labels, lse, ctx.bias32, c0, V, smoothing, ignore_index, skip)  # skipped -> 0
            _dh_accumulate(dh, lg, wc)
            with torch.no_grad():
                if gw is not None:
                    wgrad_accumulate(gw[c0:c0 + n], lg, h, async_ok=False, defer=False)  # tied: embed bwd adds too
                elif dw is not None:
                    dw[c0:c0 + n] += torch.mm(lg.t(), h)
        if p is not None:
            _fire(p)
        return dh.to(h.dtype), (dw.to(w.dtype) if dw is not None else None), None, None, None, None, None


class _LMHeadCEFusedFn(torch.autograd.Function):
    """LM head + CE with the CE inside the GEMM epilogues (module docstring, GEMM-fused variant)."""

    @staticmethod
    def forward(ctx, h, w, bias, labels, smoothing, ignore_index, params):
        C = _ext.native()
        bias32 = bias.float().reshape(-1).contiguous() if bias is not None else None
        loss_rows, lse = C.lmhead_ce_fwd(h, w, labels, bias32, float(smoothing), int(ignore_index))
        count = (labels != ignore_index).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(h, w, labels, lse, count)
        ctx.bias32 = bias32
        ctx.cfg = (float(smoothing), int(ignore_index))
        ctx.params = params
        if params is not None:
            _use(params[0])
        return loss_rows.sum() / count

    @staticmethod
    def backward(ctx, g):
        C = _ext.native()
        h, w, labels, lse, count = ctx.saved_tensors
        smoothing, ignore_index = ctx.cfg
        N, d = h.shape
        V = w.shape[0]
        vc = _chunk_cols(N, V)
        scale = (g.float() / count).reshape(1).contiguous()
        p = ctx.params[0] if ctx.params is not None else None
        gw = _gbuf(p) if p is not None else None
        dw = torch.zeros_like(w, dtype=torch.float32) if (gw is None and ctx.needs_input_grad[1]) else None
        dh = torch.zeros(N, d, dtype=torch.float32, device=h.device)
        buf = torch.empty(N * min(vc + 8, V), dtype=h.dtype, device=h.device)
        for c0, n, skip in _chunks(V, vc):
            lg = buf[:N * n].view(N, n)
            wc = w[c0:c0 + n]
            C.lmhead_ce_bwd_slice(h, wc, labels, lse, scale, ctx.bias32, lg, c0, V, smoothing, ignore_index, skip)
            _dh_accumulate(dh, lg, wc)
            with torch.no_grad():
                if gw is not None:
                    wgrad_accumulate(gw[c0:c0 + n], lg, h, async_ok=False, defer=False)  # tied: embed bwd adds too
                elif dw is not None:
                    dw[c0:c0 + n] += torch.mm(lg.t(), h)
        if p is not None:
            _fire(p)
        return dh.to(h.dtype), (dw.to(w.dtype) if dw is not None else None), None, None, None, None, None


def use_fused() -> bool:
    """The GEMM-epilogue CE (``_LMHeadCEFusedFn``) in place of the vocabulary-chunked path.  ops/routing.py ``lmhead``:
    ``auto`` (default) = whenever logits are not materialised (it beats the chunked path: no logits round trip, no CE
    passes); ``fused`` = also below the full-logits budget; ``logits`` = never.  Below the budget the materialised-logits path
    stays the default: it skips the backward's logits recompute and was 1.0 % faster per t5-base b=512 step
    (profiles/r4_lmhead_fused_ab.txt)."""
    return routing.get("lmhead") != "logits"


def fused_ok(h: torch.Tensor, w: torch.Tensor) -> bool:
    """Shapes the GEMM-epilogue CE handles (csrc/bind.cpp check_lmhead_operands): bf16, d % 64 == 0, 16-B rows."""
    return (use_fused() and h.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and h.shape[-1] % 64 == 0
            and w.stride(-1) == 1 and w.stride(0) % 8 == 0 and w.data_ptr() % 16 == 0 and h.data_ptr() % 16 == 0
            and _ext.use_native(h))


def lm_head_loss(hidden: torch.Tensor, weight: torch.Tensor, labels: torch.Tensor, *, scale: float | None = None,
                 bias: torch.Tensor | None = None, label_smoothing: float = 0.0, ignore_index: int = -100):
    """Mean (label-smoothed) CE of ``(hidden * scale) @ weightᵀ (+ bias)`` against ``labels`` over non-ignored rows,
    computed in vocabulary chunks (module docstring).  ``hidden [..., d]``, ``labels [...]``."""
    d = hidden.shape[-1]
    h = hidden.reshape(-1, d)
    if scale is not None:
        h = h * scale
    lab = labels.reshape(-1)
    if not _ext.use_native(h) or h.dtype != torch.bfloat16:  # the chunk kernels take bf16 logits; fp32: composite
        return _reference(h, weight, lab, bias, label_smoothing, ignore_index)
    params = None
    w = weight
    if torch.is_grad_enabled() and _fusable(weight) and weight.requires_grad:
        params = (weight,)
        w = weight.detach()
    h = h.contiguous()
    if fused_ok(h, w):
        return _LMHeadCEFusedFn.apply(h, w, bias, lab.contiguous(), label_smoothing, ignore_index, params)
    return _LMHeadCEFn.apply(h, w, bias, lab.contiguous(), label_smoothing, ignore_index, params)
