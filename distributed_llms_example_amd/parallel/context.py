"""Context parallelism: ring attention over a CP process group.

The reference never scales sequence length: it truncates inputs to 1024 tokens
(ref/train-accelerator.py:115-127, ref/train-task.py:157-168) and HF T5 materialises an O(S^2·H) float
bias (dep/transformers/integrations/sdpa_attention.py:150-152).  For the long-sequence flan-t5-xl config
of BASELINE.json this module shards the ENCODER sequence over ``W`` ranks of a CP group.  Everything in
the encoder except attention is per-token and runs on the local shard unchanged; attention becomes a
ring:

* forward: every rank keeps its query shard and passes its K/V shard (one packed ``[2,B,S,H,D]`` buffer)
  to the next rank W-1 times over point-to-point sends (RCCL p2p over the direct xGMI link between the
  two GPUs; gloo on CPU), starting the next transfer before computing the current block.  Each block
  runs the flash forward kernel (csrc/attn.hip) and returns (o_blk, lse_blk); blocks merge by their
  log-sum-exp (kernel LSE is in log2 units).
* backward: the flash backward kernel runs per block with the GLOBAL o / lse, so dQ accumulates locally
  while the K/V shard travels the ring together with its fp32 dK/dV accumulator; one final hop delivers
  dK/dV to the owner.
* T5 relative bias: the bias of block (q shard r, kv shard s) is the bucket table indexed by GLOBAL
  distance, i.e. ``relative_bias_lut(table, S, S, ..., q_offset=(r - s)·S)`` — W small ``[H, 2S-1]``
  LUTs, differentiable into the table.
* attention dropout: each (q shard, kv shard) block draws its keep mask from its own seed
  (``seed ^ block-hash``), which the backward regenerates exactly; the masks differ from the unsharded
  op's, as any two dropout draws do.

Weight gradients of a CP rank are partial sums over its tokens, so the data-parallel gradient reducer
just reduces over all ranks (DP × CP) with the loss normalised by the global token count.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from .. import _ext
from ..ops.attention import relative_bias_lut

_LN2 = math.log(2.0)


# --------------------------------------------------------------------------- per-block compute


def _block_seed(seed: int, qi: int, kj: int) -> int:
    return (int(seed) ^ ((qi * 0x9E3779B1 + kj * 0x85EBCA77 + 0x27D4EB2F) & 0x7FFFFFFF)) & 0x7FFFFFFF


def _ref_scores(q, k, kpm, lut, scale):
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    s = torch.matmul(q.float().permute(0, 2, 1, 3), k.float().permute(0, 2, 3, 1)) * scale
    if lut is not None:
        rel = torch.arange(Sk, device=q.device)[None, :] - torch.arange(Sq, device=q.device)[:, None] + (Sq - 1)
        s = s + lut.float()[:, rel].unsqueeze(0)
    if kpm is not None:
        s = s.masked_fill(~kpm.bool()[:, None, None, :], float("-inf"))
    return s


def _ref_block_fwd(q, k, v, kpm, lut, scale, p, seed):
    """Plain-torch block forward: (o fp32 [B,Sq,H,D], lse [B,H,Sq] in log2 units, +inf = no key)."""
    from ..ops.rng import attention_keep_mask
    B, Sq, H, D = q.shape
    s = _ref_scores(q, k, kpm, lut, scale)
    lse = torch.logsumexp(s, dim=-1)
    lse = torch.where(torch.isneginf(lse), torch.full_like(lse, float("inf")), lse)
    pr = torch.exp(s - lse.unsqueeze(-1))
    if p > 0.0:
        pr = pr * attention_keep_mask(seed, p, B, H, Sq, k.shape[1], q.device).to(pr.dtype) / (1.0 - p)
    o = torch.matmul(pr, v.float().permute(0, 2, 1, 3)).permute(0, 2, 1, 3)
    return o, lse / _LN2


def _ref_block_bwd(do, q, k, v, o, lse2, kpm, lut, scale, p, seed, need_dlut):
    from ..ops.rng import attention_keep_mask
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    s = _ref_scores(q, k, kpm, lut, scale)
    pr = torch.exp(s - (lse2 * _LN2).unsqueeze(-1))  # +inf lse -> 0
    dof = do.float().permute(0, 2, 1, 3)
    vf = v.float().permute(0, 2, 1, 3)
    delta = (do.float() * o.float()).sum(-1).permute(0, 2, 1)  # [B,H,Sq]
    dpd = torch.matmul(dof, vf.transpose(-1, -2))
    if p > 0.0:
        keep = attention_keep_mask(seed, p, B, H, Sq, Sk, q.device).to(pr.dtype) / (1.0 - p)
        pd, dp = pr * keep, dpd * keep
    else:
        pd, dp = pr, dpd
    ds = pr * (dp - delta.unsqueeze(-1))
    dq = torch.matmul(ds, k.float().permute(0, 2, 1, 3)).permute(0, 2, 1, 3) * scale
    dk = torch.matmul(ds.transpose(-1, -2), q.float().permute(0, 2, 1, 3)).permute(0, 2, 1, 3) * scale
    dv = torch.matmul(pd.transpose(-1, -2), dof).permute(0, 2, 1, 3)
    dlut = None
    if need_dlut:
        rel = (torch.arange(Sk, device=q.device)[None, :] - torch.arange(Sq, device=q.device)[:, None] + (Sq - 1))
        dlut = torch.zeros(H, Sq + Sk - 1, device=q.device, dtype=torch.float32)
        dlut.index_add_(1, rel.reshape(-1), ds.sum(0).reshape(H, -1))
    return dq, dk, dv, dlut


def _block_fwd(q, k, v, kpm, lut, sat, scale, p, seed):
    if _ext.use_native(q):
        C = _ext.native()
        lo, hi = sat if sat is not None else (-1, -1)
        o, lse, dmask = C.attn_fwd(q, k, v, kpm, lut, float(scale), False, float(p), int(seed), None, lo, hi)
        return o, lse, dmask  # bf16: the fp32 merge promotes (no separate conversion kernels)
    o, lse = _ref_block_fwd(q, k, v, kpm, lut, scale, p, seed)
    return o, lse, None


def _block_bwd(do, q, k, v, o, lse, kpm, lut, sat, scale, p, seed, need_dlut, dmask):
    if _ext.use_native(q):
        C = _ext.native()
        lo, hi = sat if sat is not None else (-1, -1)
        dq, dk, dv, dlut = C.attn_bwd(do, q, k, v, o, lse, kpm, lut, float(scale), False, float(p), int(seed),
                                      bool(need_dlut), None, None, None, dmask, lo, hi)
        return dq, dk, dv, dlut  # bf16; accumulated into fp32 buffers by promoting in-place adds
    return _ref_block_bwd(do, q, k, v, o, lse, kpm, lut, scale, p, seed, need_dlut)


def _merge(o_acc, lse_acc, o_blk, lse_blk):
    """Combine two partial softmax-attention results by their log2-sum-exp (+inf = empty)."""
    a = torch.where(torch.isinf(lse_acc), torch.full_like(lse_acc, float("-inf")), lse_acc)
    b = torch.where(torch.isinf(lse_blk), torch.full_like(lse_blk, float("-inf")), lse_blk)
    m = torch.maximum(a, b)
    m_safe = torch.where(torch.isneginf(m), torch.zeros_like(m), m)
    wa, wb = torch.exp2(a - m_safe), torch.exp2(b - m_safe)
    tot = wa + wb
    lse = torch.where(tot > 0, m_safe + torch.log2(tot.clamp_min(1e-38)), torch.full_like(m, float("inf")))
    inv = torch.where(tot > 0, 1.0 / tot.clamp_min(1e-38), torch.zeros_like(tot))
    fa = (wa * inv).permute(0, 2, 1).unsqueeze(-1)  # [B,H,Sq] -> [B,Sq,H,1]
    fb = (wb * inv).permute(0, 2, 1).unsqueeze(-1)
    return o_acc * fa + o_blk * fb, lse


# --------------------------------------------------------------------------- ring transport


class _Ring:
    def __init__(self, group):
        self.group = group
        on = dist.is_available() and dist.is_initialized()
        self.W = dist.get_world_size(group) if on else 1
        self.r = dist.get_rank(group) if on else 0
        glob = (lambda i: dist.get_global_rank(group, i)) if group is not None else (lambda i: i)
        self.nxt = glob((self.r + 1) % self.W) if self.W > 1 else self.r
        self.prv = glob((self.r - 1) % self.W) if self.W > 1 else self.r

    def start(self, send: torch.Tensor):
        """Send ``send`` to the next rank, receive the previous rank's buffer; returns (recv, works)."""
        recv = torch.empty_like(send)
        ops = [dist.P2POp(dist.isend, send, self.nxt, self.group), dist.P2POp(dist.irecv, recv, self.prv, self.group)]
        return recv, dist.batch_isend_irecv(ops)

    @staticmethod
    def wait(works):
        for w in works:
            w.wait()


class _RingAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, luts, kpm_full, sats, scale, p, seed, group):
        ring = _Ring(group)
        W, r = ring.W, ring.r
        S = k.shape[1]
        kv = torch.stack([k, v]).contiguous()
        o_acc = lse_acc = None
        dmasks = [None] * W
        for step in range(W):
            src = (r - step) % W
            nxt_kv = works = None
            if step < W - 1:
                nxt_kv, works = ring.start(kv)
            kpm = kpm_full[:, src * S:(src + 1) * S].contiguous() if kpm_full is not None else None
            lut = luts[src] if luts is not None else None
            sat = sats[src] if sats is not None else None
            o_b, lse_b, dmasks[src] = _block_fwd(q, kv[0], kv[1], kpm, lut, sat, scale, p, _block_seed(seed, r, src))
            if o_acc is None:
                o_acc, lse_acc = o_b, lse_b
            else:
                o_acc, lse_acc = _merge(o_acc, lse_acc, o_b, lse_b)
            if works is not None:
                ring.wait(works)
                kv = nxt_kv
        o = o_acc.to(q.dtype)
        ctx.save_for_backward(q, k, v, o, lse_acc.contiguous(), luts, kpm_full)
        ctx.cfg = (sats, scale, p, seed, group, luts is not None and luts.requires_grad)
        ctx.dmasks = dmasks
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, luts, kpm_full = ctx.saved_tensors
        sats, scale, p, seed, group, need_dlut = ctx.cfg
        dmasks, ctx.dmasks = ctx.dmasks, None
        ring = _Ring(group)
        W, r = ring.W, ring.r
        S = k.shape[1]
        do = do.contiguous()
        kv = torch.stack([k, v]).contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        dluts = torch.zeros_like(luts) if need_dlut else None
        dkv_in = dworks = sending = None
        for step in range(W):
            src = (r - step) % W
            nxt_kv = works = None
            if step < W - 1:  # the K/V shard moves on while this block computes
                nxt_kv, works = ring.start(kv)
            kpm = kpm_full[:, src * S:(src + 1) * S].contiguous() if kpm_full is not None else None
            lut = luts[src] if luts is not None else None
            sat = sats[src] if sats is not None else None
            dq_b, dk_b, dv_b, dlut_b = _block_bwd(do, q, kv[0], kv[1], o, lse, kpm, lut, sat, scale, p,
                                                  _block_seed(seed, r, src), need_dlut, dmasks[src])
            dq += dq_b
            if need_dlut:
                dluts[src] += dlut_b
            if dworks is None:
                acc = torch.stack([dk_b, dv_b]).float()
            else:  # this shard's fp32 dK/dV accumulator, sent by the previous rank during this block
                ring.wait(dworks)
                acc = dkv_in
                acc[0] += dk_b
                acc[1] += dv_b
            if W > 1:  # pass it on; the transfer overlaps the next block's compute
                sending = acc
                dkv_in, dworks = ring.start(sending)
            if works is not None:
                ring.wait(works)
                kv = nxt_kv
        if W > 1:
            ring.wait(dworks)
            acc = dkv_in
        dkv = acc
        del sending
        # after W hops the accumulator that arrived belongs to this rank's own K/V shard
        return (dq.to(q.dtype), dkv[0].to(k.dtype), dkv[1].to(v.dtype), dluts, None, None, None, None, None, None)


def ring_attention(q, k, v, *, group=None, scale: float = 1.0, key_padding_mask=None, bias_table=None,
                   bidirectional: bool = True, num_buckets: int = 32, max_distance: int = 128,
                   dropout_p: float = 0.0, seed: int = 0):
    """Bidirectional (encoder) attention over a sequence sharded contiguously across ``group``.

    q/k/v: this rank's shard ``[B, S, H, D]`` (global positions ``rank·S .. rank·S+S-1``);
    key_padding_mask: this rank's ``[B, S]`` bool (True = attend), all-gathered once;
    bias_table: T5 relative-attention bucket table ``[num_buckets, H]`` (differentiable) or None.
    Returns this rank's output shard ``[B, S, H, D]``."""
    on = dist.is_available() and dist.is_initialized()
    W = dist.get_world_size(group) if on else 1
    r = dist.get_rank(group) if on else 0
    S = q.shape[1]
    assert k.shape[1] == S and v.shape[1] == S, "ring_attention: equal-length shards required"
    kpm_full = None
    if key_padding_mask is not None:
        m = key_padding_mask.to(torch.uint8).contiguous()
        if W > 1:
            parts = [torch.empty_like(m) for _ in range(W)]
            dist.all_gather(parts, m, group=group)
            m = torch.cat(parts, 1)
        kpm_full = m.contiguous()
    luts = sats = None
    if bias_table is not None:
        ls = [relative_bias_lut(bias_table, S, S, bidirectional, num_buckets, max_distance, q_offset=(r - s) * S)
              for s in range(W)]
        sats = [lt._dllm_sat for lt in ls]
        luts = torch.stack(ls)
    return _RingAttnFn.apply(q, k, v, luts, kpm_full, sats, float(scale), float(dropout_p), int(seed), group)


# --------------------------------------------------------------------------- model glue


def _cp_world(group):
    on = dist.is_available() and dist.is_initialized()
    return (dist.get_world_size(group) if on else 1), (dist.get_rank(group) if on else 0)


def shard_sequence(t: torch.Tensor | None, group=None, dim: int = 1):
    """This rank's contiguous slice of a ``[B, S, ...]`` tensor (S must divide by the CP size)."""
    if t is None:
        return None
    W, r = _cp_world(group)
    S = t.shape[dim]
    assert S % W == 0, f"context parallel: sequence length {S} not divisible by {W} ranks"
    return t.narrow(dim, r * (S // W), S // W)


class _GatherSeq(torch.autograd.Function):
    """All-gather the encoder output along the sequence.  Every rank of the CP group runs the SAME decoder on
    the gathered tensor, so the incoming gradients are identical across ranks; the backward keeps this
    rank's slice scaled by W, which after the data-parallel reducer's average over ranks equals the sum of
    the per-shard encoder gradients (no communication in backward)."""

    @staticmethod
    def forward(ctx, x, group):
        W, r = _cp_world(group)
        ctx.cfg = (W, r, x.shape[1])
        if W == 1:
            return x
        parts = [torch.empty_like(x) for _ in range(W)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, 1)

    @staticmethod
    def backward(ctx, g):
        W, r, S = ctx.cfg
        if W == 1:
            return g, None
        return g.narrow(1, r * S, S) * W, None


def context_parallel_encode(encode_fn, input_ids, attention_mask, group=None):
    """Run ``encode_fn`` on this rank's sequence shard and return (full encoder output, full mask).

    The encoder draws its dropout seeds from a per-shard stream (outer seed mixed with the CP rank); the
    outer stream advances identically on every CP rank, so the decoder's dropout masks agree across the
    group as _GatherSeq requires."""
    from ..ops.rng import default_rng, mix_host, rng_scope
    W, r = _cp_world(group)
    s = default_rng().next_seed()
    with rng_scope(mix_host(s, 1 + r)):
        enc_local = encode_fn(input_ids, attention_mask)
    enc = _GatherSeq.apply(enc_local, group)
    mask = attention_mask
    if mask is not None and W > 1:
        parts = [torch.empty_like(mask) for _ in range(W)]
        dist.all_gather(parts, mask.contiguous(), group=group)
        mask = torch.cat(parts, 1)
    return enc, mask


# --------------------------------------------------------------------------- single-GPU long sequences


class _ChunkedAttnFn(torch.autograd.Function):
    """The ring's block algorithm inside one process: a (Wq x Wk) grid of C x C flash-attention blocks merged by
    LSE.  The single-kernel path stages per-key state and the bias window in LDS, which bounds it to ~8K keys
    (csrc/attn.hip launch checks); chunking lifts that bound for long encoders on one GPU, and 4K-token blocks
    measured faster per FLOP than one 8K kernel (profiles/r1_cp_attention_bench.jsonl).  ``luts[d + W - 1]``
    is the LUT of block offset d = qi - kj."""

    @staticmethod
    def forward(ctx, q, k, v, luts, kpm, sats, C, Cq, scale, p, seed):
        W, Wq = k.shape[1] // C, q.shape[1] // Cq
        outs, lses, dmasks = [], [], {}
        for qi in range(Wq):
            qs = q[:, qi * Cq:(qi + 1) * Cq]
            o_acc = l_acc = None
            for kj in range(W):
                d = qi - kj + W - 1
                km = kpm[:, kj * C:(kj + 1) * C].contiguous() if kpm is not None else None
                o_b, l_b, dmasks[(qi, kj)] = _block_fwd(qs, k[:, kj * C:(kj + 1) * C], v[:, kj * C:(kj + 1) * C], km,
                                                        luts[d] if luts is not None else None,
                                                        sats[d] if sats is not None else None, scale, p,
                                                        _block_seed(seed, qi, kj))
                o_acc, l_acc = (o_b, l_b) if o_acc is None else _merge(o_acc, l_acc, o_b, l_b)
            outs.append(o_acc.to(q.dtype))
            lses.append(l_acc.contiguous())
        o = torch.cat(outs, 1)
        ctx.save_for_backward(q, k, v, o, torch.stack(lses), luts, kpm)
        ctx.cfg = (sats, C, Cq, scale, p, seed, luts is not None and luts.requires_grad)
        ctx.dmasks = dmasks
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lses, luts, kpm = ctx.saved_tensors
        sats, C, Cq, scale, p, seed, need_dlut = ctx.cfg
        dmasks, ctx.dmasks = ctx.dmasks, None
        W, Wq = k.shape[1] // C, q.shape[1] // Cq
        do = do.contiguous()
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        dk = torch.zeros(k.shape, dtype=torch.float32, device=k.device)
        dv = torch.zeros(v.shape, dtype=torch.float32, device=v.device)
        dluts = torch.zeros_like(luts) if need_dlut else None
        for qi in range(Wq):
            sq = slice(qi * Cq, (qi + 1) * Cq)
            do_q, o_q = do[:, sq].contiguous(), o[:, sq].contiguous()
            for kj in range(W):
                sk = slice(kj * C, (kj + 1) * C)
                d = qi - kj + W - 1
                km = kpm[:, sk].contiguous() if kpm is not None else None
                a, b, c, dl = _block_bwd(do_q, q[:, sq], k[:, sk], v[:, sk], o_q, lses[qi], km,
                                         luts[d] if luts is not None else None, sats[d] if sats is not None else None,
                                         scale, p, _block_seed(seed, qi, kj), need_dlut, dmasks[(qi, kj)])
                dq[:, sq] += a
                dk[:, sk] += b
                dv[:, sk] += c
                if need_dlut:
                    dluts[d] += dl
        return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), dluts, None, None, None, None, None, None, None


def _pad_seq(x, n):
    """[B, S, ...] zero-padded at the end of the sequence dim to length n."""
    S = x.shape[1]
    if S == n:
        return x
    return torch.cat([x, x.new_zeros((x.shape[0], n - S) + tuple(x.shape[2:]))], 1)


def _padded_kpm(key_padding_mask, B, S, n, device):
    """uint8 key mask for a sequence padded from S to n keys (the padding is masked out), or None."""
    if key_padding_mask is None and n == S:
        return None
    kpm = (key_padding_mask.to(torch.uint8) if key_padding_mask is not None
           else torch.ones(B, S, dtype=torch.uint8, device=device))
    return _pad_seq(kpm, n).contiguous()


def chunked_cross_attention(q, k, v, *, chunk: int, scale: float = 1.0, key_padding_mask=None,
                            dropout_p: float = 0.0, seed: int = 0):
    """Cross-attention (no bias, not causal) of a short query over a long key sequence in ``chunk``-key blocks
    (decoder over a long encoder output).  A key length that is not a multiple of ``chunk`` is padded with
    masked keys (ragged last block)."""
    Sk = k.shape[1]
    n = -(-Sk // chunk) * chunk
    kpm = _padded_kpm(key_padding_mask, k.shape[0], Sk, n, k.device)
    return _ChunkedAttnFn.apply(q, _pad_seq(k, n), _pad_seq(v, n), None, kpm, None, int(chunk), int(q.shape[1]),
                                float(scale), float(dropout_p), int(seed))


def chunked_attention(q, k, v, *, chunk: int, scale: float = 1.0, key_padding_mask=None, bias_table=None,
                      bidirectional: bool = True, num_buckets: int = 32, max_distance: int = 128,
                      dropout_p: float = 0.0, seed: int = 0):
    """Bidirectional self-attention over a long sequence on one device in ``chunk``-token blocks.  Same arguments
    as :func:`ring_attention`.  A length that is not a multiple of ``chunk`` is padded at the end (padded keys
    masked, padded query rows dropped; real tokens keep their positions, so the relative bias is unchanged)."""
    N0 = q.shape[1]
    assert k.shape[1] == N0, "chunked_attention: self-attention needs equal query / key lengths"
    N = -(-N0 // chunk) * chunk
    if N != N0:
        kpm = _padded_kpm(key_padding_mask, q.shape[0], N0, N, q.device)
        o = chunked_attention(_pad_seq(q, N), _pad_seq(k, N), _pad_seq(v, N), chunk=chunk, scale=scale,
                              key_padding_mask=kpm, bias_table=bias_table, bidirectional=bidirectional,
                              num_buckets=num_buckets, max_distance=max_distance, dropout_p=dropout_p, seed=seed)
        return o[:, :N0]
    W = N // chunk
    luts = sats = None
    if bias_table is not None:
        ls = [relative_bias_lut(bias_table, chunk, chunk, bidirectional, num_buckets, max_distance,
                                q_offset=(d - (W - 1)) * chunk) for d in range(2 * W - 1)]
        sats = [lt._dllm_sat for lt in ls]
        luts = torch.stack(ls)
    kpm = key_padding_mask.to(torch.uint8).contiguous() if key_padding_mask is not None else None
    return _ChunkedAttnFn.apply(q, k, v, luts, kpm, sats, int(chunk), int(chunk), float(scale), float(dropout_p),
                                int(seed))


def long_sequence_chunk(n: int, cross: bool = False, rows: int = 0) -> int | None:
    """Chunk size for an encoder of ``n`` tokens, or None when the single kernel handles it
    (ops/routing.py ``attn_chunk`` = block length, default 4096, used above ``attn_chunk_min`` = 8192 tokens;
    -1 disables).  ``rows`` = batch x heads: with fewer than 32 rows a 4K block launches under 1024 query-tile
    workgroups (4 per CU), so the default block grows to 8K.  Cross-attention (a short query: few workgroups per block) keeps the single kernel up to
    its 16K-key limit and then uses 16K-key blocks."""
    from ..ops import routing
    c = int(routing.get("attn_chunk")) or (8192 if 0 < rows < 32 else 4096)
    lo = int(routing.get("attn_chunk_min"))
    if cross and c > 0 and lo >= 8192:  # (test overrides with a small attn_chunk_min chunk cross too)
        c, lo = max(c, 16384), max(lo, 16384)
    if c <= 0 or n <= max(lo, c):
        return None
    # ceil(n / c) blocks of equal length (a multiple of 128, the kernels' query tile); chunked_attention pads the
    # sequence to blocks x chunk with masked keys, so any n (primes too) keeps blocks near c
    w = -(-n // c)
    g = min(128, c)
    return -(-n // (w * g)) * g
