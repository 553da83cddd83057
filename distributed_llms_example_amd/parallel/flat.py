"""Flat parameter / gradient storage.

Every trainable parameter becomes a view into ONE contiguous parameter buffer and its gradient a
view into ONE contiguous gradient buffer (``p.grad`` when the buffer has the parameter dtype; with
fp32 gradients for bf16 weights — the default of train/engine.py, matching the reference's fp32
gradients — ``p._dllm_gbuf``, which the fused ops accumulate into), laid out in reverse registration order (≈ the order in
which backward produces gradients).  This is the memory layout the whole runtime is built on:

* the gradient reducer (parallel/reducer.py) all-reduces contiguous slices of the gradient buffer
  in place — "gradient as bucket view", the layout torch DDP's C++ Reducer builds per bucket
  (torch/nn/parallel/distributed.py:828-834, reducer.cpp) — with no flatten/unflatten copies;
* the fused AdamW (ops/optim.py) runs ONE kernel over the whole buffer instead of a multi-tensor
  launch group, and the clip-grad norm is one reduction (transformers trainer.py:2535-2539 →
  torch clip_grad.py:93-96 does foreach norms over ~500 tensors);
* train-task's per-tensor ``all_reduce`` loop (ref/train-task.py:65-69) becomes one coalesced
  all-reduce over the same bytes.

Segments are padded to 64 elements so every parameter starts 128-byte aligned for the vector
loads in csrc/adamw.hip.  Tied parameters (T5 ``shared`` == ``lm_head``) appear once.
"""
from __future__ import annotations

import builtins
from dataclasses import dataclass

import torch
import torch.nn as nn

ALIGN = 64
builtins_range = builtins.range


@dataclass
class Segment:
    name: str
    offset: int
    numel: int
    shape: tuple


class FlatParams:
    def __init__(self, module: nn.Module, grad_dtype: torch.dtype | None = None, reverse: bool = True):
        seen = set()
        named = []
        for n, p in module.named_parameters():
            if not p.requires_grad or id(p) in seen:
                continue
            seen.add(id(p))
            named.append((n, p))
        if reverse:
            named = named[::-1]
        # parameters a fused op consumes as ONE stacked tensor (ops/linear.py stacked_linear, e.g. the
        # decoder's per-layer cross-attention K/V weights) are placed back-to-back, in group order,
        # where the group's first member would have gone
        groups = module._dllm_param_groups() if hasattr(module, "_dllm_param_groups") else []
        self.groups: list[list[int]] = []  # id()s of each stacked group, kept adjacent by relayout() too
        for grp in groups:
            ids = [id(p) for p in grp]
            pos = {id(p): i for i, (_, p) in enumerate(named)}
            if not all(i in pos for i in ids):
                continue
            self.groups.append(ids)
            first = min(pos[i] for i in ids)
            members = {id(p): (n, p) for n, p in named if id(p) in ids}
            rest = [(n, p) for n, p in named if id(p) not in members]
            at = sum(1 for n, p in named[:first] if id(p) not in members)
            named = rest[:at] + [members[i] for i in ids] + rest[at:]
        if not named:
            raise ValueError("module has no trainable parameters")
        dtypes = {p.dtype for _, p in named}
        devices = {p.device for _, p in named}
        if len(dtypes) != 1 or len(devices) != 1:
            raise ValueError(f"FlatParams needs one dtype/device, got {dtypes} {devices}")
        self.dtype = dtypes.pop()
        self.device = devices.pop()
        self.grad_dtype = grad_dtype or self.dtype
        self.segments: list[Segment] = []
        self.params: list[nn.Parameter] = []
        off = 0
        for n, p in named:
            self.segments.append(Segment(n, off, p.numel(), tuple(p.shape)))
            self.params.append(p)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self._companions: list[tuple[object, str]] = []  # flat-indexed tensors kept in step with relayout()
        self.canonical = [s.name for s in self.segments]  # construction order (optimizer state is saved in it)
        self.param_buf = torch.zeros(off, dtype=self.dtype, device=self.device)
        self.grad_buf = torch.zeros(off, dtype=self.grad_dtype, device=self.device)
        # autograd insists p.grad has p's dtype: with fp32 gradients for bf16 weights the flat slices are handed
        # to the fused ops as p._dllm_gbuf instead, and p.grad stays None
        self.views_as_grad = self.grad_dtype == self.dtype
        self._hooks = []
        with torch.no_grad():
            for i, (seg, p) in enumerate(zip(self.segments, self.params)):
                view = self.param_buf[seg.offset:seg.offset + seg.numel].view(seg.shape)
                view.copy_(p.data)
                p.data = view
                # ops/linear.py may accumulate this parameter's weight gradient inside the GEMM
                p._dllm_fused_wgrad = True
                p._dllm_gbuf = self.grad_view(i)
                p._dllm_pending = 0
                p._dllm_fused_seen = False
                self._hooks.append(p.register_post_accumulate_grad_hook(self._autograd_hook))
        self.attach_grads()

    # -------------------------------------------------------------------------------------------
    def grad_view(self, i: int) -> torch.Tensor:
        seg = self.segments[i]
        return self.grad_buf[seg.offset:seg.offset + seg.numel].view(seg.shape)

    @staticmethod
    def _autograd_hook(p) -> None:
        """A gradient that arrived through ordinary autograd (AccumulateGrad: e.g. T5's relative-position
        bias table): fold it into the flat buffer when ``p.grad`` is not the flat slice itself (fp32 buffer,
        or a user-replaced .grad), then run the reducer hooks like the fused ops do (ops/linear.py)."""
        g = p.grad
        gb = p._dllm_gbuf
        if getattr(p, "_dllm_fused_seen", False):
            raise RuntimeError(f"parameter {tuple(p.shape)} receives gradients both from fused ops and from autograd; route all of "
                               "its uses through ops.linear / ops.embedding (or none)")
        if g is not None and g.data_ptr() != gb.data_ptr():
            gb.add_(g)
            p.grad = gb if gb.dtype == p.dtype else None
        for h in getattr(p, "_dllm_post_hooks", ()):
            h(p)

    def attach_grads(self) -> None:
        """(Re)bind every ``p.grad`` to its slice of the flat gradient buffer (same-dtype buffer only)."""
        for i, p in enumerate(self.params):
            p.grad = self.grad_view(i) if self.views_as_grad else None

    def reset_pending(self) -> None:
        """Forget fused-use counts of a forward that never ran backward (ops/linear.py ``_use``)."""
        for p in self.params:
            p._dllm_pending = 0
            p._dllm_fused_seen = False

    def zero_grad(self) -> None:
        self.grad_buf.zero_()
        self.reset_pending()
        # something (e.g. user code) may have replaced a .grad: re-bind cheaply
        for i, p in enumerate(self.params):
            g = p.grad
            if not self.views_as_grad:
                if g is not None:
                    p.grad = None
            elif g is None or g.data_ptr() != self.grad_buf.data_ptr() + self.segments[i].offset * self.grad_buf.element_size():
                p.grad = self.grad_view(i)

    # ------------------------------------------------------------------------------------------- layout
    def register_companion(self, obj, attr: str) -> None:
        """``getattr(obj, attr)`` is indexed like the flat buffers (optimizer master weights / moments, weight-decay
        mask): relayout() permutes it together with the parameters."""
        self._companions.append((obj, attr))

    def _offsets(self, order: list[int]) -> tuple[list[int], int]:
        offs, off = [0] * len(self.segments), 0
        for i in order:
            offs[i] = off
            off += (self.segments[i].numel + ALIGN - 1) // ALIGN * ALIGN
        return offs, off

    def _permute(self, t: torch.Tensor, src_offs: list[int], dst_offs: list[int], n: int) -> torch.Tensor:
        out = torch.zeros(n, dtype=t.dtype, device=t.device)
        for i, seg in enumerate(self.segments):
            out[dst_offs[i]:dst_offs[i] + seg.numel] = t[src_offs[i]:src_offs[i] + seg.numel]
        return out

    @torch.no_grad()
    def relayout(self, order: list[int]) -> None:
        """Re-lay the flat buffers with segment ``order[0]`` first, ``order[1]`` next, ... (the reducer's observed
        gradient-ready order, parallel/reducer.py).  Parameters, gradients (values kept) and every registered
        companion buffer move together; parameter views and gradient slices are re-pointed."""
        assert sorted(order) == list(builtins_range(len(self.segments))), "order must be a permutation of segments"
        order = self.keep_groups_adjacent(order)
        src = [seg.offset for seg in self.segments]
        dst, n = self._offsets(order)
        self.param_buf = self._permute(self.param_buf, src, dst, n)
        self.grad_buf = self._permute(self.grad_buf, src, dst, n)
        for obj, attr in self._companions:
            t = getattr(obj, attr)
            if t is not None:
                setattr(obj, attr, self._permute(t, src, dst, n))
        segs = [Segment(self.segments[i].name, dst[i], self.segments[i].numel, self.segments[i].shape) for i in order]
        params = [self.params[i] for i in order]
        self.segments, self.params, self.numel = segs, params, n
        for i, (seg, p) in enumerate(zip(self.segments, self.params)):
            p.data = self.param_buf[seg.offset:seg.offset + seg.numel].view(seg.shape)
            p._dllm_gbuf = self.grad_view(i)
        self.attach_grads()
        # a stacked group that is no longer one block would send ops/linear.py stacked_linear to its slow torch.cat
        # path on every forward (same results): fail here instead
        idx = {id(p): i for i, p in enumerate(self.params)}
        for ids in self.groups:
            at = [idx[i] for i in ids]
            assert at == list(builtins_range(at[0], at[0] + len(at))), f"stacked parameter group split by relayout: {at}"

    def keep_groups_adjacent(self, order: list[int]) -> list[int]:
        """``order`` with every stacked group's members moved back-to-back (in group order) to where its first
        member appears: the reducer's ready order interleaves them whenever another hook fires in between."""
        if not self.groups:
            return list(order)
        seg_of = {id(p): i for i, p in enumerate(self.params)}
        member = {}
        for gi, ids in enumerate(self.groups):
            for i in ids:
                member[seg_of[i]] = gi
        out, placed = [], set()
        for i in order:
            gi = member.get(i)
            if gi is None:
                out.append(i)
            elif gi not in placed:
                placed.add(gi)
                out.extend(seg_of[j] for j in self.groups[gi])
        return out

    def canonical_offsets(self) -> tuple[list[int], list[int], int]:
        """(current offsets, canonical offsets, canonical numel) per current segment."""
        pos = {name: i for i, name in enumerate(self.canonical)}
        order = sorted(builtins_range(len(self.segments)), key=lambda i: pos[self.segments[i].name])
        can, n = self._offsets(order)
        return [seg.offset for seg in self.segments], can, n

    def to_canonical(self, t: torch.Tensor) -> torch.Tensor:
        cur, can, n = self.canonical_offsets()
        return t if cur == can else self._permute(t, cur, can, n)

    def from_canonical(self, t: torch.Tensor) -> torch.Tensor:
        cur, can, n = self.canonical_offsets()
        return t if cur == can else self._permute(t, can, cur, self.numel)

    def grads(self) -> list[torch.Tensor]:
        """Per-parameter gradient views of the flat buffer (fp32 or param dtype), in ``params`` order."""
        return [self.grad_view(i) for i in range(len(self.params))]

    def decay_mask(self, no_decay_pred) -> torch.Tensor | None:
        """uint8 mask over the flat buffer: 1 where weight decay applies; None if uniform."""
        flags = [0 if no_decay_pred(s.name) else 1 for s in self.segments]
        if all(flags) or not any(flags):
            return None
        m = torch.zeros(self.numel, dtype=torch.uint8, device=self.device)
        for s, f in zip(self.segments, flags):
            if f:
                m[s.offset:s.offset + s.numel] = 1
        return m

    def state_layout(self) -> list[dict]:
        return [{"name": s.name, "offset": s.offset, "numel": s.numel, "shape": list(s.shape)} for s in self.segments]
