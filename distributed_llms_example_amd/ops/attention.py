"""Fused multi-head attention for encoder-decoder models (flash-style, HIP/MFMA on gfx950).

One op covers every attention variant the reference's models run (SURVEY.md §2.3 "SDPA attention"):

* T5 self-attention: no 1/sqrt(d) scale (transformers modeling_t5.py:196-197) and an additive
  relative-position bias built from a (num_buckets, H) table (modeling_t5.py:217-279).  HF
  materialises the bias as a float ``[1, H, Sq, Sk]`` mask, which also knocks SDPA off its flash path
  (integrations/sdpa_attention.py:39-76).  Here the bias is a per-head LUT indexed by the relative
  distance ``j - i`` (``[H, Sq + Sk - 1]``, O(S) memory) that the kernel reads from LDS; its
  backward returns the gradient of that LUT (diagonal sums of dS), which autograd scatters back
  into the bucket table.
* T5 / BART decoder: causal (+ bias); cross-attention: key-padding mask only.
* BART: scale ``d**-0.5`` (modeling_bart.py:169), key-padding mask.
* Attention-probability dropout (T5 applies ``dropout_rate`` to the probabilities,
  modeling_t5.py:360) with the counter-based mask of ops/rng.py, regenerated in backward.

Layout: q ``[B, Sq, H, D]``, k/v ``[B, Sk, H, D]`` — the natural output of the fused QKV GEMM
viewed without any transpose copy (only the last dim must be contiguous).  Output ``[B, Sq, H, D]``.

Kernels: csrc/attn.hip (bf16: forward; backward = dQ kernel + dK/dV kernel, no atomics except the bias LUT) and
csrc/attn_f32.hip (fp32, the reference's own precision: the same op on the f32-input matrix cores, O(S) memory).
"""
from __future__ import annotations

import math


import torch

from .. import _ext
from . import routing
from . import streams
from .gemm import colsum_record
from .rng import attention_keep_mask

# --------------------------------------------------------------------------- T5 relative bias


def relative_position_bucket(relative_position: torch.Tensor, bidirectional: bool = True, num_buckets: int = 32,
                             max_distance: int = 128) -> torch.Tensor:
    """Bit-exact re-statement of T5Attention._relative_position_bucket (modeling_t5.py:217-262)."""
    relative_buckets = 0
    if bidirectional:
        num_buckets //= 2
        relative_buckets += (relative_position > 0).to(torch.long) * num_buckets
        relative_position = torch.abs(relative_position)
    else:
        relative_position = -torch.min(relative_position, torch.zeros_like(relative_position))
    max_exact = num_buckets // 2
    is_small = relative_position < max_exact
    rp_large = max_exact + (torch.log(relative_position.float() / max_exact) / math.log(max_distance / max_exact)
                            * (num_buckets - max_exact)).to(torch.long)
    rp_large = torch.min(rp_large, torch.full_like(rp_large, num_buckets - 1))
    relative_buckets += torch.where(is_small, relative_position, rp_large)
    return relative_buckets


_bucket_cache: dict = {}


def relative_bias_lut(table: torch.Tensor, q_len: int, k_len: int, bidirectional: bool, num_buckets: int,
                      max_distance: int, q_offset: int = 0) -> torch.Tensor:
    """Per-head bias indexed by relative distance: ``lut[h, (j - i) + (q_len - 1)]`` for local query
    row ``i`` (absolute position ``i + q_offset``) and key ``j``.  Differentiable w.r.t. ``table``
    (shape ``[num_buckets, H]``).  Returns fp32 ``[H, q_len + k_len - 1]``."""
    key = (q_len, k_len, bidirectional, num_buckets, max_distance, q_offset, table.device)
    hit = _bucket_cache.get(key)
    if hit is None:
        rel = torch.arange(-(q_len - 1), k_len, dtype=torch.long) - q_offset
        idx = relative_position_bucket(rel, bidirectional, num_buckets, max_distance)
        hit = (idx.to(table.device), saturated_ranges(idx))
        if len(_bucket_cache) > 256:
            _bucket_cache.clear()
        _bucket_cache[key] = hit
    idx, sat = hit
    lut = table.float().index_select(0, idx).t().contiguous()
    # the kernels may treat tiles inside these constant-bucket ranges as scalar-bias tiles (csrc/attn_params.h):
    # valid because this LUT's gradient only reaches the table through index_select (per bucket)
    lut._dllm_sat = sat
    return lut


def saturated_ranges(idx: torch.Tensor) -> tuple[int, int]:
    """(sat_lo, sat_hi) for a bucket index row over the LUT: entries [0, sat_lo] share idx[0]'s bucket and
    [sat_hi, L) share idx[-1]'s (T5 buckets saturate at +-max_distance)."""
    L = idx.numel()
    same_lo = (idx == idx[0]).long().cumprod(0).sum().item()
    same_hi = (idx.flip(0) == idx[-1]).long().cumprod(0).sum().item()
    if same_lo == L:  # one bucket everywhere (far-apart context-parallel shards): all of it is the low range
        return L - 1, L
    return int(same_lo) - 1, int(L - same_hi)


# --------------------------------------------------------------------------- reference


def _reference(q, k, v, scale, causal, kpm, lut, p, seed):
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    qf = q.float().permute(0, 2, 1, 3)
    kf = k.float().permute(0, 2, 1, 3)
    vf = v.float().permute(0, 2, 1, 3)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if lut is not None:
        rel = torch.arange(Sk, device=q.device)[None, :] - torch.arange(Sq, device=q.device)[:, None] + (Sq - 1)
        s = s + lut.float()[:, rel].unsqueeze(0)
    neg = torch.finfo(torch.float32).min
    if kpm is not None:
        s = s.masked_fill(~kpm.bool()[:, None, None, :], neg)
    if causal:
        off = Sk - Sq
        cm = torch.arange(Sk, device=q.device)[None, :] > (torch.arange(Sq, device=q.device)[:, None] + off)
        s = s.masked_fill(cm, neg)
    pr = torch.softmax(s, dim=-1)
    if p > 0.0:
        keep = attention_keep_mask(seed, p, B, H, Sq, Sk, q.device)
        pr = pr * keep.to(pr.dtype) * (1.0 / (1.0 - p))
    o = torch.matmul(pr, vf)
    return o.permute(0, 2, 1, 3).to(q.dtype)


# --------------------------------------------------------------------------- native


def _split(mode, a, b, c):
    if mode == "qkv":  # a = [B,S,3,H,D]
        return a[:, :, 0], a[:, :, 1], a[:, :, 2]
    if mode == "q_kv":  # a = q, b = [B,Sk,2,H,D]
        return a, b[:, :, 0], b[:, :, 1]
    return a, b, c


class _AttnFn(torch.autograd.Function):
    """Inputs are packed the way the projections produce them (``qkv`` = one [B,S,3,H,D] tensor for
    self-attention, ``q`` + ``kv`` [B,Sk,2,H,D] for cross-attention) so backward writes ONE packed
    gradient buffer through strided views instead of three zero-padded slice gradients."""

    @staticmethod
    def forward(ctx, mode, a, b, c, lut, kpm, scale, causal, p, seed, pre=None):
        C = _ext.native()
        q, k, v = _split(mode, a, b, c)
        if q.dtype == torch.float32:  # csrc/attn_f32.hip
            o, lse = C.attn_f32_fwd(q, k, v, kpm, lut, float(scale), bool(causal), float(p), int(seed))
            ctx.save_for_backward(a, b, c, o, lse, lut, kpm, None)
            ctx.cfg = (mode, scale, causal, p, seed, lut is not None and lut.requires_grad, -1, -1)
            ctx.grad_into = getattr(b, "_dllm_grad_into", None) if mode == "q_kv" else None
            return o
        dmask_in = None
        if pre is not None:  # keep-bit planes generated ahead on the side stream (prefetch_dropout_mask)
            dmask_in, ev = pre
            cur = torch.cuda.current_stream(q.device)
            cur.wait_event(ev)
            dmask_in.record_stream(cur)
        sat = getattr(lut, "_dllm_sat", None) if lut is not None else None
        sat_lo, sat_hi = sat if sat is not None else (-1, -1)
        # saturated bias tiles add a scalar instead of reading the LUT (forward -2 %)
        o, lse, dmask = C.attn_fwd(q, k, v, kpm, lut, float(scale), bool(causal), float(p), int(seed), dmask_in,
                                   sat_lo, sat_hi)
        ctx.save_for_backward(a, b, c, o, lse, lut, kpm, dmask)
        ctx.cfg = (mode, scale, causal, p, seed, lut is not None and lut.requires_grad, sat_lo, sat_hi)
        # packed inputs straight from a biased projection (ops/linear.py marks its output): the backward kernels also
        # sum dQ / dK / dV over tokens for that projection's bias gradient (colsum_record)
        # (bias-LUT-free calls only: the kernels' column-sum variants exist for those, csrc/attn.hip)
        cs_ok = BIAS_COLSUM and lut is None
        ctx.cs = (cs_ok and mode != "sep" and _bias_out(a), cs_ok and mode == "q_kv" and _bias_out(b))
        # ops/linear.py stacked_linear: the packed kv is a slice of a multi-layer projection and its
        # gradient has a home in the stacked gradient buffer — write dK/dV there directly
        ctx.grad_into = getattr(b, "_dllm_grad_into", None) if mode == "q_kv" else None
        return o

    @staticmethod
    def backward(ctx, do):
        C = _ext.native()
        a, b, c, o, lse, lut, kpm, dmask = ctx.saved_tensors
        mode, scale, causal, p, seed, need_dlut, sat_lo, sat_hi = ctx.cfg
        q, k, v = _split(mode, a, b, c)
        da = db = dc = None
        if mode == "qkv":
            da = torch.empty_like(a)
            dq, dk, dv = da[:, :, 0], da[:, :, 1], da[:, :, 2]
        elif mode == "q_kv":
            da = torch.empty_like(a)
            gi = ctx.grad_into
            db = gi if gi is not None and gi.shape == b.shape else torch.empty_like(b)
            ctx.grad_into = None
            dq, dk, dv = da, db[:, :, 0], db[:, :, 1]
        else:
            dq = dk = dv = None
        part = pq = pkv = None
        csq = csk = csv = None
        if q.dtype != torch.float32 and (ctx.cs[0] or ctx.cs[1]):
            B, Sq, H = q.shape[0], q.shape[1], q.shape[2]
            HD, nq, nk = H * 64, B * ((Sq + 127) // 128), B * ((k.shape[1] + 127) // 128)
            f32 = dict(device=q.device, dtype=torch.float32)
            if mode == "qkv":  # one [blocks, 3 H D] buffer: the q | k | v thirds of the fused bias
                part = torch.empty(nq, 3 * HD, **f32)
                csq, csk, csv = part[:, :HD], part[:, HD:2 * HD], part[:, 2 * HD:]
            else:
                if ctx.cs[0]:
                    pq = csq = torch.empty(nq, HD, **f32)
                if ctx.cs[1]:
                    pkv = torch.empty(nk, 2 * HD, **f32)
                    csk, csv = pkv[:, :HD], pkv[:, HD:]
        if q.dtype == torch.float32:
            rq, rk, rv, dlut = C.attn_f32_bwd(do.contiguous(), q, k, v, o, lse, kpm, lut, float(scale), bool(causal),
                                              float(p), int(seed), bool(need_dlut), dq, dk, dv)
        else:
            rq, rk, rv, dlut = C.attn_bwd(do.contiguous(), q, k, v, o, lse, kpm, lut, float(scale), bool(causal),
                                          float(p), int(seed), bool(need_dlut), dq, dk, dv, dmask, sat_lo, sat_hi,
                                          csq, csk, csv)
        if part is not None:  # per-block partials, reduced by the consumer into the bias gradient (ops/gemm.py)
            colsum_record(da, part)
        if pq is not None:
            colsum_record(da, pq)
        if pkv is not None:
            colsum_record(db, pkv)
        if mode == "sep":
            da, db, dc = rq, rk, rv
        streams.pair_join()  # side-stream weight gradients paired with these VALU-bound kernels (ops/streams.py)
        return None, da, db, dc, (dlut if need_dlut else None), None, None, None, None, None, None


# False: the projections' bias gradients from a separate column reduction of dQKV (tests flip the module attribute)
BIAS_COLSUM = True


def _bias_out(t) -> bool:
    """t (or the tensor it is a full view of) is a biased projection's output (ops/linear.py ``_dllm_bias_out``)."""
    if t is None:
        return False
    if getattr(t, "_dllm_bias_out", False):
        return True
    src = t._base
    return (src is not None and getattr(src, "_dllm_bias_out", False) and src.data_ptr() == t.data_ptr()
            and src.numel() == t.numel())


def _prep_kpm(kpm):
    if kpm is not None and kpm.dtype != torch.uint8:
        kpm = kpm.to(torch.uint8)
    return kpm.contiguous() if kpm is not None else None


def _native(t) -> bool:
    """bf16 -> csrc/attn.hip; fp32 — the reference's own precision (ref/train-torchrun.py:115-128 sets neither bf16
    nor fp16; Accelerate's default mixed_precision is 'no') — -> csrc/attn_f32.hip (f32-input MFMA, exact f32
    products).  Head dim 64 (every model this framework builds).  Anything else (CPU, other head dims) takes the
    composite ``_reference`` below, the exact-math oracle the kernels are tested against.  ops/routing.py ``attn_f32``
    = 0 sends fp32 to the composite (A/B)."""
    if not _ext.use_native(t) or t.shape[-1] != 64:
        return False
    if t.dtype == torch.bfloat16:
        return True
    return t.dtype == torch.float32 and bool(routing.get("attn_f32"))


def attention(q, k, v, *, scale: float = 1.0, causal: bool = False, key_padding_mask=None, bias_lut=None,
              dropout_p: float = 0.0, seed: int = 0):
    """Multi-head attention.  q ``[B,Sq,H,D]``, k/v ``[B,Sk,H,D]``; ``key_padding_mask`` bool
    ``[B,Sk]`` (True = attend); ``bias_lut`` from :func:`relative_bias_lut`."""
    if _native(q):
        return _AttnFn.apply("sep", q, k, v, bias_lut, _prep_kpm(key_padding_mask), scale, causal, dropout_p, seed)
    return _reference(q, k, v, scale, causal, key_padding_mask, bias_lut, dropout_p, seed)


def attention_qkv(qkv, pre=None, **kw):
    """Self-attention on the fused projection output ``qkv`` = [B, S, 3, H, D]."""
    if _native(qkv):
        return _AttnFn.apply("qkv", qkv, None, None, kw.get("bias_lut"), _prep_kpm(kw.get("key_padding_mask")),
                             kw.get("scale", 1.0), kw.get("causal", False), kw.get("dropout_p", 0.0), kw.get("seed", 0),
                             pre)
    return attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], **kw)


_SIDE: dict = {}


def prefetch_dropout_mask(like: torch.Tensor, B: int, H: int, Sq: int, Sk: int, p: float, seed: int):
    """Generate the attention-dropout keep bits for an upcoming call on a side HIP stream (the VALU-only mask kernel
    overlapping a projection GEMM issued meanwhile on the compute stream).  Returns a handle for
    ``attention_qkv(pre=...)`` or None.  Not used by the models: the forward hashing the bits itself measured faster
    (profiles/r3_attn_dropout_packed_ab.txt); kept as an API, tested equal to the in-kernel bits."""
    if p <= 0.0 or not _native(like) or like.dtype != torch.bfloat16:
        return None
    dev = like.device
    side = _SIDE.get(dev)
    if side is None:
        side = _SIDE[dev] = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        m = _ext.native().attn_dropout_mask(B, H, Sq, Sk, float(p), int(seed), like)
        ev = torch.cuda.Event()
        ev.record(side)
    return m, ev


def attention_q_kv(q, kv, **kw):
    """Cross-attention with q = [B, Sq, H, D] and the fused key/value projection kv = [B, Sk, 2, H, D]."""
    if _native(q):
        return _AttnFn.apply("q_kv", q, kv, None, kw.get("bias_lut"), _prep_kpm(kw.get("key_padding_mask")),
                             kw.get("scale", 1.0), kw.get("causal", False), kw.get("dropout_p", 0.0), kw.get("seed", 0))
    return attention(q, kv[:, :, 0], kv[:, :, 1], **kw)
