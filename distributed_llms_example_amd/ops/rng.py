"""Counter-based dropout RNG shared by the HIP kernels and the torch reference path.

Every dropout site gets a 32-bit ``seed`` from :class:`DropoutRNG`; element ``i`` of the tensor is
kept iff the 16-bit half ``i & 1`` of ``mix32(seed, i >> 1)`` is ``>= threshold16(p)`` — one hash
serves two adjacent elements (half the VALU cost inside the attention / norm kernels; p is quantised
to 1/65536).  Because the decision is a pure function of
(seed, index), backward kernels regenerate the mask instead of storing it (no mask tensors in HBM),
and the reference implementation below reproduces the kernels' masks bit-for-bit so numerics tests
can run with p > 0.  Mirrors csrc/common.h ``dllm_mix32``.

Kernels that walk rows — attention probabilities and the FFN activations — draw their decisions from the row-Weyl
hash instead (:func:`rowwise_keep_mask`, csrc/common.h ``rw_*``): one ``mix32`` per row, then ~7 full-rate VALU per
column pair, where ``mix32`` per pair costs three quarter-rate 32-bit multiplies (the T5 ReLU FFN forward epilogue:
dropout 290 -> 160 us at the t5-base b=512 shape, profiles/r6_ffn_rowweyl_dropout_ab.txt).  The flat-index hash
stays for the residual dropout of the norm kernels and the standalone dropout kernel (memory-bound).
"""
from __future__ import annotations

import torch

_C1 = 0x9E3779B1
_M1 = 0x85EBCA6B
_M2 = 0xC2B2AE35
_MASK = 0xFFFFFFFF


def mix32(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """murmur3-fmix32 of (idx * golden) ^ seed, computed in int64 with 32-bit wraparound."""
    x = ((idx.to(torch.int64) * _C1) & _MASK) ^ (seed & _MASK)
    x = x ^ (x >> 16)
    x = (x * _M1) & _MASK
    x = x ^ (x >> 13)
    x = (x * _M2) & _MASK
    x = x ^ (x >> 16)
    return x


def threshold16(p: float) -> int:
    return min(int(p * 65536.0), 0xFFFF)


def keep_from_index(seed: int, p: float, idx: torch.Tensor) -> torch.Tensor:
    """Keep decision for element indices ``idx`` (any shape, int64)."""
    h = mix32(effective_seed(seed), idx >> 1)
    half = torch.where((idx & 1) == 1, h >> 16, h & 0xFFFF)
    return half >= threshold16(p)


def keep_mask(seed: int, p: float, shape, device, numel_offset: int = 0) -> torch.Tensor:
    """Boolean keep-mask of ``shape`` (row-major element indices starting at ``numel_offset``)."""
    n = 1
    for s in shape:
        n *= s
    idx = torch.arange(numel_offset, numel_offset + n, device=device, dtype=torch.int64)
    return keep_from_index(seed, p, idx).view(shape)


_G = 0x9E3779B1
_C24 = 0x9E3779
_C24B = 0x85EBCB


def rowwise_keep_mask(seed: int, p: float, rows: int, cols: int, device, row0: int = 0) -> torch.Tensor:
    """Keep mask [rows, cols] of the row-Weyl hash (mirrors csrc/common.h ``rw_gbase`` / ``rw_pair_y`` / ``rw_drop2``),
    the decisions of the kernels that walk rows: attention probabilities (one row per (b, h, query)) and the T5 ReLU FFN
    activation (one row per token).

    Per row ``r`` (``row0`` + 0 .. rows-1): ``rh = mix32(seed, r)`` (computed once per row in the kernels); per column
    pair ``kp = j >> 1``: ``g = (rh & 0xFFFFFF) * C24 + kp * G`` (mod 2^32: a Weyl sequence along the row, one add per
    pair in the kernels), ``h = ((g ^ (g >> 15)) & 0xFFFFFF) * C24B`` (the xorshift + multiply round: ``g`` alone is
    linear in ``kp`` and leaves lag-2 drops anti-correlated), ``y = h ^ (h >> 16)``; the even column keeps iff
    ``(y & 0xFFFF) ^ 0x8000 >= threshold16(p)``, the odd column iff ``(y >> 16) ^ 0x8000 >= threshold16(p)`` (the
    kernels compare both halves at once as signed 16-bit values)."""
    r = torch.arange(row0, row0 + rows, device=device, dtype=torch.int64)
    rh = mix32(effective_seed(seed), r).view(rows, 1)
    j = torch.arange(cols, device=device, dtype=torch.int64).view(1, cols)
    g = ((rh & 0xFFFFFF) * _C24 + (j >> 1) * _G) & _MASK
    h = (((g ^ (g >> 15)) & 0xFFFFFF) * _C24B) & _MASK
    y = h ^ (h >> 16)
    half = torch.where((j & 1) == 1, y >> 16, y & 0xFFFF)
    return (half ^ 0x8000) >= threshold16(p)


def attention_keep_mask(seed: int, p: float, B: int, H: int, Sq: int, Sk: int, device) -> torch.Tensor:
    """Attention-probability mask [B, H, Sq, Sk] (csrc/attn.hip): :func:`rowwise_keep_mask` with one row per
    query of each (batch, head), ``r = (b*H + h)*Sq + i``."""
    return rowwise_keep_mask(seed, p, B * H * Sq, Sk, device).view(B, H, Sq, Sk)


def mix_host(seed: int, idx: int) -> int:
    x = ((idx * _C1) & _MASK) ^ (seed & _MASK)
    x ^= x >> 16
    x = (x * _M1) & _MASK
    x ^= x >> 13
    x = (x * _M2) & _MASK
    x ^= x >> 16
    return x


class DropoutRNG:
    """Per-process seed stream.  ``next_seed()`` is called once per dropout site per forward; the
    seed is saved for the backward.  ``state_dict`` makes resumed runs reproduce the stream.

    Step-seed mode (``StepSeed``, for HIP-graph replay): the kernels mix a DEVICE step counter into every site seed,
    so the host stream restarts at the same point every micro-step (``begin_micro_step``) — the seeds a captured graph
    baked in are exactly the ones an eager step would draw, and the masks still change every step."""

    def __init__(self, seed: int = 42):
        self.base = seed & _MASK
        self.counter = 0
        self.site_mode = False

    def next_seed(self) -> int:
        self.counter += 1
        return mix_host(self.base, self.counter)

    def begin_micro_step(self):
        if self.site_mode:
            self.counter = 0

    def state_dict(self):
        return {"base": self.base, "counter": self.counter}

    def load_state_dict(self, d):
        self.base = int(d["base"])
        self.counter = int(d["counter"])


class StepSeed:
    """Device step counter mixed into every dropout site seed by the HIP kernels (csrc/common.h DLLM_SEED_STEP_TU):
    effective seed = mix32(site seed, step).  ``advance()`` is a device add (captured by a graph, so each replay draws
    new masks); ``host`` mirrors it for the reference ops and for checkpoints (no device read)."""

    def __init__(self, device, start: int = 0):
        self.t = torch.full((1,), start, dtype=torch.int32, device=device)
        self.host = start
        self.enabled = False
        self._prev_site_mode = None

    def enable(self):
        """Process-wide: the kernels' step pointer (every translation unit), the active-step registry read by the
        reference ops, and the host seed stream's site mode.  ``disable()`` restores all three."""
        from .. import _ext
        if self.t.is_cuda and _ext.native() is not None:
            _ext.native().set_seed_step(self.t)
        self.enabled = True
        _active_step[0] = self
        rng = default_rng()
        if self._prev_site_mode is None:
            self._prev_site_mode = rng.site_mode
        rng.site_mode = True

    def disable(self):
        from .. import _ext
        if self.t.is_cuda and _ext.native() is not None:
            _ext.native().set_seed_step(None)
        self.enabled = False
        if _active_step[0] is self:
            _active_step[0] = None
        if self._prev_site_mode is not None:
            default_rng().site_mode = self._prev_site_mode
            self._prev_site_mode = None

    def advance(self, n: int = 1):
        self.t.add_(n)
        self.host += n


_active_step: list = [None]


def effective_seed(seed: int) -> int:
    """The seed a kernel actually hashes with (the reference ops mirror it): the site seed, mixed with the device step
    counter's host mirror in step-seed mode."""
    st = _active_step[0]
    if st is None or not st.enabled:
        return seed
    return mix_host(seed & _MASK, st.host & _MASK)


_global = DropoutRNG(42)
_scoped: list[DropoutRNG] = []


def default_rng() -> DropoutRNG:
    return _scoped[-1] if _scoped else _global


class rng_scope:
    """Run a region with its own seed stream derived from ``seed``.  Every transformer block draws one seed
    from the outer stream and runs under ``rng_scope(seed)``, so activation checkpointing can recompute a
    block in backward with bit-identical dropout masks (the outer stream is not replayed)."""

    def __init__(self, seed: int):
        self.rng = DropoutRNG(seed)

    def __enter__(self):
        _scoped.append(self.rng)
        return self.rng

    def __exit__(self, *exc):
        _scoped.pop()
        return False


def manual_seed(seed: int) -> None:
    _global.base = seed & _MASK
    _global.counter = 0
