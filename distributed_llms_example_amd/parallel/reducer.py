"""Bucketed data-parallel gradient reducer on RCCL (torch.distributed "nccl" backend on ROCm).

Replaces torch DDP's C++ Reducer that the reference reaches through HF Trainer / Accelerate
(torch/nn/parallel/distributed.py:828-834,1227-1251 → reducer.cpp) and train-task's per-tensor loop
(ref/train-task.py:65-69), built on the flat gradient buffer (parallel/flat.py):

* buckets are contiguous slices of ONE gradient buffer ("gradient as bucket view"): all-reduce runs
  in place, no flatten/unflatten copies;
* a bucket is launched (``all_reduce(AVG, async_op=True)``) from the post-accumulate-grad hook of its
  last parameter, in bucket order on every rank, so RCCL runs on its own stream while the rest of
  backward computes (overlap); ``finish()`` (queued at the end of backward) launches leftovers and
  makes the compute stream wait on the RCCL work — no host synchronisation;
* bucket sizing for MI355X: a ring all-reduce over xGMI is per-link bound (≈153 GB/s per link,
  7 links per GPU), so buckets are much larger than DDP's 25 MiB default (the launch/latency cost
  per bucket, not link bandwidth, dominates small buckets); the first bucket stays small (1 MiB,
  DDP's ``_DEFAULT_FIRST_BUCKET_BYTES``) so communication starts early in backward;
* ``no_sync()`` for gradient accumulation (HF Trainer trainer.py:1750-1757);
* ``overlap=False`` → one coalesced all-reduce after backward (train-task semantics, same math).

Two engines implement the same bucket/launch policy: the native one (csrc/reducer.cpp,
``NativeReducer``: bucket state machine and c10d ``ProcessGroup::allreduce`` launches in C++ — the
counterpart of DDP's C++ Reducer; readiness is signalled per parameter by FlatParams' post-accumulate
hooks and by the fused ops, ops/linear.py ``_fire``) is used whenever the
extension is built (``DLLM_NATIVE_REDUCER=0`` selects the Python engine below, kept as the readable
reference and for A/B tests).  Bucket layout is computed here once and handed to either engine.
"""
from __future__ import annotations

import contextlib

import os

import torch
import torch.distributed as dist

from .. import _ext
from .flat import FlatParams

DEFAULT_BUCKET_MB = 128.0
FIRST_BUCKET_MB = 1.0


class GradReducer:
    def __init__(self, flat: FlatParams, group=None, bucket_mb: float = DEFAULT_BUCKET_MB,
                 first_bucket_mb: float = FIRST_BUCKET_MB, overlap: bool = True, average: bool = True,
                 native: bool | None = None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(group) if dist.is_initialized() else "none"
        self.overlap = overlap
        self.average = average
        self.enabled = True
        esz = flat.grad_buf.element_size()
        self.buckets: list[tuple[int, int]] = []
        self.seg_bucket: list[int] = []
        limit = min(first_bucket_mb, bucket_mb) * 2**20
        start = flat.segments[0].offset
        cur_bytes = 0
        counts = []
        n_in = 0
        for i, seg in enumerate(flat.segments):
            seg_end = flat.segments[i + 1].offset if i + 1 < len(flat.segments) else flat.numel
            cur_bytes += (seg_end - seg.offset) * esz
            self.seg_bucket.append(len(self.buckets))
            n_in += 1
            if cur_bytes >= limit or i + 1 == len(flat.segments):
                self.buckets.append((start, seg_end))
                counts.append(n_in)
                start = seg_end
                cur_bytes = 0
                n_in = 0
                limit = bucket_mb * 2**20
        self._counts = counts
        self._pending = list(counts)
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._works = []
        self._callback_queued = False
        self._hooks = []
        self._manual = []
        self.native = None
        if native is None:
            native = os.environ.get("DLLM_NATIVE_REDUCER", "1") != "0" and _ext.native() is not None
        if native and self.world > 1:
            pg = group if group is not None else dist.distributed_c10d._get_default_group()
            bounds = [x for se in self.buckets for x in se]
            self.native = _ext.native().NativeReducer(flat.grad_buf, bounds, self.seg_bucket, pg, average,
                                                      self.backend == "nccl")
            if overlap:  # readiness comes from FlatParams' hooks / the fused ops (ops/linear.py _fire)
                for i, p in enumerate(flat.params):
                    p._dllm_post_hooks = getattr(p, "_dllm_post_hooks", []) + [
                        (lambda _q, i=i, nat=self.native: nat.mark_ready(i))]
                    self._manual.append(p)
        elif self.world > 1 and overlap:
            for i, p in enumerate(flat.params):
                h = self._make_hook(i)
                # run by FlatParams' post-accumulate hook (autograd gradients) or by the fused op that accumulated
                # the gradient in its kernel (ops/linear.py _fire), once per backward after the last contribution
                p._dllm_post_hooks = getattr(p, "_dllm_post_hooks", []) + [h]
                self._manual.append(p)

    # --------------------------------------------------------------------------------- hooks
    def _make_hook(self, seg_index: int):
        def hook(_p):
            if not self.enabled:
                return
            if not self._callback_queued:
                self._callback_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self.finish)
            b = self.seg_bucket[seg_index]
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._ready[b] = True
                self._launch_ready()
        return hook

    def _launch(self, b: int):
        s, e = self.buckets[b]
        view = self.flat.grad_buf[s:e]
        if self.average and self.backend == "nccl":
            w = dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        else:
            w = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._works.append((b, w))

    def _launch_ready(self):
        while self._next < len(self.buckets) and self._ready[self._next]:
            self._launch(self._next)
            self._next += 1

    def finish(self):
        """End of backward: launch what is left (unused params) in order, wait on the GPU stream."""
        if self.world <= 1:
            return
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        for _, w in self._works:
            w.wait()
        if self.average and self.backend != "nccl":
            self.flat.grad_buf.div_(self.world)
        self._works.clear()
        self._pending = list(self._counts)
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._callback_queued = False

    # --------------------------------------------------------------------------------- API
    @contextlib.contextmanager
    def no_sync(self):
        prev = self.enabled
        self.enabled = False
        if self.native is not None:
            self.native.set_enabled(False)
        try:
            yield
        finally:
            self.enabled = prev
            if self.native is not None:
                self.native.set_enabled(prev)

    def sync_now(self):
        """Non-overlapped path (train-task semantics): one coalesced all-reduce of all gradients."""
        if self.world <= 1:
            return
        if self.native is not None:
            self.native.sync_all()
            return
        g = self.flat.grad_buf
        if self.average and self.backend == "nccl":
            dist.all_reduce(g, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
            if self.average:
                g.div_(self.world)

    def post_backward(self):
        """Call after ``loss.backward()``: completes the reduction for the non-overlapped mode."""
        if self.world > 1 and not self.overlap and self.enabled:
            self.sync_now()

    def broadcast_params(self, module=None, src: int = 0):
        """DDP construction broadcast (distributed.py:864-870): one collective over the flat
        parameter buffer plus the module's buffers."""
        if self.world <= 1:
            return
        dist.broadcast(self.flat.param_buf, src=src, group=self.group)
        if module is not None:
            for b in module.buffers():
                dist.broadcast(b.data, src=src, group=self.group)

    def bucket_sizes_mb(self) -> list[float]:
        esz = self.flat.grad_buf.element_size()
        return [(e - s) * esz / 2**20 for s, e in self.buckets]

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
        for p in self._manual:
            p._dllm_post_hooks = []
        self._manual.clear()
        if self.native is not None:
            self.native.detach()
