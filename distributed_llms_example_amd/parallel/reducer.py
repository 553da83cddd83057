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
* ``overlap=False`` → one coalesced all-reduce after backward (train-task semantics, same math);
* ``wire_dtype=torch.bfloat16`` (``--grad-reduce-dtype bf16``) → compress for the wire only: gradients accumulate in
  the fp32 flat buffer, each bucket is cast to a persistent bf16 shadow on the compute stream at launch, all-reduced
  in bf16 (half the bytes over xGMI) and widened back into the fp32 bucket once its all-reduce has been waited for;
* segmented HIP-graph capture (train/graph.py "overlap"): ``begin_capture_cuts`` counts readiness without launching
  anything and calls back when the next bucket(s) in order became ready, so the backward graph is cut there and the
  replay launches those buckets between the segments (``launch_upto``).

Two engines implement the same bucket/launch policy: the native one (csrc/reducer.cpp,
``NativeReducer``: bucket state machine and c10d ``ProcessGroup::allreduce`` launches in C++ — the
counterpart of DDP's C++ Reducer; readiness is signalled per parameter by FlatParams' post-accumulate
hooks and by the fused ops, ops/linear.py ``_fire``) is used whenever the
extension is built (ops/routing.py ``reducer`` = python selects the Python engine below, kept as the readable
reference and for A/B tests).  Bucket layout is computed here once and handed to either engine.
"""
from __future__ import annotations

import contextlib
import time

import torch
import torch.distributed as dist

from .. import _ext
from ..ops import routing
from ..utils import profiling
from .flat import FlatParams

DEFAULT_BUCKET_MB = 128.0
FIRST_BUCKET_MB = 1.0
BUCKET_MB_CANDIDATES = (32.0, 64.0, 128.0, 256.0)


def wire_dtype_of(name: str | None) -> torch.dtype | None:
    """``--grad-reduce-dtype``: None / "fp32" -> all-reduce the fp32 buckets as they are, "bf16" -> compress-for-wire."""
    if name in (None, "", "fp32", "float32", "none"):
        return None
    if name in ("bf16", "bfloat16"):
        return torch.bfloat16
    raise ValueError(f"grad reduce dtype must be fp32 or bf16, got {name!r}")


def choose_bucket_mb(device: torch.device, total_mb: float, group=None, wire_dtype: torch.dtype | None = None,
                     candidates=BUCKET_MB_CANDIDATES, iters: int = 10, tolerance: float = 0.95,
                     warmup: int = 3) -> dict:
    """Bucket size from an in-run all-reduce probe on the job's own process group (every rank runs it: collective).

    For each candidate size (capped by the gradient buffer) the slowest rank's time of ``iters`` all-reduces of that
    many bytes (in the wire dtype), after ``warmup`` untimed ones (a cold RCCL communicator sets up its channels on the
    first calls), is measured; the bus bandwidth 2(N-1)/N x bytes / time is what RCCL over xGMI delivers
    at that size.  Chosen: the SMALLEST candidate within ``tolerance`` of the best bandwidth — large enough that the
    per-collective latency is amortised, no larger, so the first bucket launches early in backward and the exposed
    tail (the last bucket, launched when backward ends) stays short.  Returns {"bucket_mb", "busbw_gbps": {...}}."""
    n = dist.get_world_size(group)
    esz_wire = 2 if wire_dtype == torch.bfloat16 else 4
    cands = sorted({float(c) for c in candidates if c <= max(total_mb, min(candidates))})
    table = {}
    for mb in cands:
        x = torch.ones(max(1, int(mb * 2**20) // 4 * 4 // esz_wire), device=device,
                       dtype=torch.bfloat16 if wire_dtype == torch.bfloat16 else torch.float32)
        for _ in range(max(1, warmup)):
            dist.all_reduce(x, group=group)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x, group=group)
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64,
                         device=device if device.type == "cuda" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        table[mb] = 2 * (n - 1) / n * x.numel() * x.element_size() / t.item() / 1e9
    best = max(table.values())
    pick = min(mb for mb, bw in table.items() if bw >= tolerance * best)
    return {"bucket_mb": pick, "busbw_gbps": {f"{mb:g}": round(bw, 2) for mb, bw in table.items()},
            "rule": f"smallest within {tolerance:g} of the best bus bandwidth", "iters": iters, "warmup": warmup}


class GradReducer:
    def __init__(self, flat: FlatParams, group=None, bucket_mb: float | str | None = DEFAULT_BUCKET_MB,
                 first_bucket_mb: float = FIRST_BUCKET_MB, overlap: bool = True, average: bool = True,
                 native: bool | None = None, rebuild: bool | None = None, force: bool = False,
                 wire_dtype: torch.dtype | None = None):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        # data parallel: more than one rank, or ``force`` (a 1-rank process group whose collectives really run: the
        # GPU tests of the RCCL launch / graph-capture paths on a one-GPU box)
        self.dp = self.world > 1 or (bool(force) and dist.is_initialized())
        self.backend = dist.get_backend(group) if dist.is_initialized() else "none"
        self.overlap = overlap
        self.average = average
        if wire_dtype is not None and wire_dtype == flat.grad_buf.dtype:
            wire_dtype = None  # the buckets are already in that dtype
        if wire_dtype not in (None, torch.bfloat16):
            raise ValueError(f"wire dtype must be None or bfloat16, got {wire_dtype}")
        self.wire_dtype = wire_dtype
        # persistent bf16 shadow of the gradient buffer (compress-for-wire): bucket b's all-reduce runs on its slice
        self.wire_buf = (torch.empty(flat.grad_buf.numel(), dtype=wire_dtype, device=flat.grad_buf.device)
                         if wire_dtype is not None and self.dp else None)
        self._cut_fn = None  # segmented graph capture (begin_capture_cuts)
        self.enabled = True
        self.bucket_choice = None
        if bucket_mb in ("auto", None):
            bucket_mb = DEFAULT_BUCKET_MB
            if self.world > 1:  # probe on the job's own process group (every rank constructs its reducer together)
                total = flat.grad_buf.numel() * flat.grad_buf.element_size() / 2**20
                dev = flat.grad_buf.device if self.backend == "nccl" else torch.device("cpu")
                self.bucket_choice = choose_bucket_mb(dev, total, group=group, wire_dtype=wire_dtype)
                bucket_mb = self.bucket_choice["bucket_mb"]
        self.bucket_mb, self.first_bucket_mb = float(bucket_mb), first_bucket_mb
        if native is None:
            native = routing.get("reducer") != "python" and _ext.native() is not None
        self.use_native = bool(native)
        # DDP's _rebuild_buckets: after the first synchronised backward the flat layout (and with it the buckets)
        # is re-laid in the order gradients actually became ready, broadcast from rank 0 so every rank agrees
        if rebuild is None:
            rebuild = bool(routing.get("rebuild_buckets"))
        self._rebuild_pending = bool(rebuild) and overlap and self.dp
        # per synchronised backward (diagnostics / tests): segment indices in readiness order, and (bucket, number of
        # segments ready at its launch) in launch order; the previous backward's logs are kept in *_last
        self.ready_log: list[int] = []
        self.launch_log: list[tuple[int, int]] = []
        self.launches = 0  # Python engine: all-reduces actually launched (tests of the eager segmented schedule)
        self.ready_log_last: list[int] = []
        self.launch_log_last: list[tuple[int, int]] = []
        self.rebuilt = False
        self.timing = False  # set_timing(): exposed-communication events around the end-of-backward wait
        self._events: list = []
        self._host_ms: list[float] = []
        self._manual = []
        self._hooks = []
        self.native = None
        self._build()
        if self.dp and overlap:
            for p in flat.params:
                # run by FlatParams' post-accumulate hook (autograd gradients) or by the fused op that accumulated
                # the gradient in its kernel (ops/linear.py _fire), once per backward after the last contribution
                p._dllm_post_hooks = getattr(p, "_dllm_post_hooks", []) + [self._on_ready]
                self._manual.append(p)

    def _build(self):
        """Buckets over the current flat layout (segment order) and the engine that launches them."""
        flat = self.flat
        esz = flat.grad_buf.element_size()
        self.buckets: list[tuple[int, int]] = []
        self.seg_bucket: list[int] = []
        self._seg_of = {id(p): i for i, p in enumerate(flat.params)}
        limit = min(self.first_bucket_mb, self.bucket_mb) * 2**20
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
                limit = self.bucket_mb * 2**20
        self._counts = counts
        self._pending = list(counts)
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._cut_next = 0
        self._works = []
        self._callback_queued = False
        if self.native is not None:
            self.native.detach()
            self.native = None
        if self.use_native and self.dp:
            pg = self.group if self.group is not None else dist.distributed_c10d._get_default_group()
            bounds = [x for se in self.buckets for x in se]
            self.native = _ext.native().NativeReducer(flat.grad_buf, bounds, self.seg_bucket, pg, self.average,
                                                      self.backend == "nccl")
            if self.wire_buf is not None:
                self.native.set_wire_buffer(self.wire_buf)

    # --------------------------------------------------------------------------------- hooks
    def _on_ready(self, p):
        if not self.enabled:
            return
        i = self._seg_of[id(p)]
        self.ready_log.append(i)
        if self._cut_fn is not None:  # segmented capture: count, never launch (nothing may run inside the capture)
            b = self.seg_bucket[i]
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._ready[b] = True
            # the cut cursor is not the launch cursor: a cut callback may launch right away (eager segmented schedule,
            # launch_upto) and that must find its buckets still unlaunched
            first = self._cut_next
            while self._cut_next < len(self.buckets) and self._ready[self._cut_next]:
                self._cut_next += 1
            if self._cut_next > first:
                cut = list(range(first, self._cut_next))
                n0 = self._launched_count()
                self._cut_fn(cut)
                # logged here unless the Python engine's _launch logged the launches the callback just made
                if self.native is not None or self._launched_count() == n0:
                    self.launch_log.extend((b, len(self.ready_log)) for b in cut)
            return
        if self.native is not None:
            before = self.native.launched()
            self.native.mark_ready(i)
            self.launch_log.extend((b, len(self.ready_log)) for b in range(before, self.native.launched()))
            return
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self.finish)
        b = self.seg_bucket[i]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._ready[b] = True
            self._launch_ready()

    @torch.no_grad()
    def maybe_rebuild(self):
        """After the first synchronised backward (gradients final and reduced): re-lay the flat buffers in the
        observed ready order (rank 0's, broadcast) and rebuild the buckets, so bucket k holds the k-th group of
        gradients to become ready and launches as soon as they are — e.g. the decoder's stacked cross-attention
        K/V weights, whose gradient only appears at the end of the decoder backward, no longer hold back the
        bucket of the decoder's last layer.  A no-op when the order already matches."""
        if not self._rebuild_pending or not self.ready_log:
            return False
        self._rebuild_pending = False
        n = len(self.flat.segments)
        seen, order = set(), []
        for i in self.ready_log:
            if i not in seen:
                seen.add(i)
                order.append(i)
        order += [i for i in range(n) if i not in seen]  # never-ready (unused) parameters last, in layout order
        t = torch.tensor(order, dtype=torch.int64, device=self.flat.device if self.backend == "nccl" else "cpu")
        dist.broadcast(t, src=dist.get_global_rank(self.group, 0) if self.group is not None else 0, group=self.group)
        order = t.tolist()
        if order == list(range(n)):
            return False
        self.flat.relayout(order)
        self._build()
        self.rebuilt = True
        return True

    def _launched_count(self) -> int:
        return self.native.launched() if self.native is not None else self.launches

    def _launch(self, b: int):
        s, e = self.buckets[b]
        view = self.flat.grad_buf[s:e]
        if self.wire_buf is not None:  # compress for the wire (widened back in finish)
            self.wire_buf[s:e].copy_(view)
            view = self.wire_buf[s:e]
        profiling.mark(f"allreduce bucket {b} ({(e - s) * view.element_size() / 2**20:.1f} MiB)")
        if self.average and self.backend == "nccl":
            w = dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        else:
            w = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._works.append((b, w))
        self.launches += 1
        self.launch_log.append((b, len(self.ready_log)))

    def _launch_ready(self):
        while self._next < len(self.buckets) and self._ready[self._next]:
            self._launch(self._next)
            self._next += 1

    def finish(self):
        """End of backward: launch what is left (unused params) in order, wait on the GPU stream."""
        if not self.dp:
            return
        ev = None
        if self.timing and self.flat.grad_buf.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        h0 = time.perf_counter()
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        for b, w in self._works:
            w.wait()
            if self.wire_buf is not None:
                s, e = self.buckets[b]
                self.flat.grad_buf[s:e].copy_(self.wire_buf[s:e])
        if ev is not None:
            ev[1].record()
            self._events.append(ev)
        elif self.timing:  # CPU (gloo) rehearsal: wait() blocks the host
            self._host_ms.append((time.perf_counter() - h0) * 1e3)
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

    def begin_capture_cuts(self, cut_fn):
        """Segmented graph capture of a synchronised backward (train/graph.py "overlap"): readiness is counted as
        usual but nothing is launched; ``cut_fn(buckets)`` is called (on the autograd thread) each time the next
        bucket(s) in bucket order became ready — the point where the capture cuts the backward graph and the replay
        launches them.  ``end_capture_cuts`` returns the buckets left for after the backward."""
        self._pending = list(self._counts)
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._cut_next = 0
        self._cut_fn = cut_fn

    def end_capture_cuts(self) -> list[int]:
        """Buckets no cut covered: launched after the backward."""
        rest = list(range(self._cut_next, len(self.buckets)))
        self._cut_fn = None
        self._pending = list(self._counts)
        self._ready = [False] * len(self.buckets)
        self._cut_next = 0
        return rest

    def launch_upto(self, n: int):
        """Launch buckets [launched, n) in order (async all-reduce; replay of a segmented graph step)."""
        if not self.dp:
            return
        if self.native is not None:
            self.native.launch_upto(n)
            return
        while self._next < min(n, len(self.buckets)):
            self._launch(self._next)
            self._next += 1

    def sync_buckets(self):
        """Every bucket, in bucket order, as an async all-reduce; then the compute stream waits on them (no host sync
        on RCCL).  The frozen launch schedule a graphed data-parallel step issues between its replays
        (train/graph.py "split"): identical on every rank by construction (``layout_signature``)."""
        if not self.dp:
            return
        if self.native is not None:
            self.native.finalize()  # launches buckets next_..end (all of them: no hook has fired), waits, resets
        else:
            self.finish()

    def sync_now(self):
        """Non-overlapped path (train-task semantics): one coalesced all-reduce of all gradients."""
        if not self.dp:
            return
        if self.native is not None:
            self.native.sync_all()
            return
        g = self.flat.grad_buf
        if self.wire_buf is not None:
            w = self.wire_buf
            w.copy_(g)
            dist.all_reduce(w, op=dist.ReduceOp.AVG if (self.average and self.backend == "nccl") else dist.ReduceOp.SUM,
                            group=self.group)
            g.copy_(w)
            if self.average and self.backend != "nccl":
                g.div_(self.world)
            return
        if self.average and self.backend == "nccl":
            dist.all_reduce(g, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
            if self.average:
                g.div_(self.world)

    def post_backward(self):
        """Call after a synchronised ``loss.backward()``: completes the reduction for the non-overlapped mode, rebuilds
        the buckets in ready order after the first one (maybe_rebuild) and rotates the readiness / launch logs."""
        if self.dp and not self.overlap and self.enabled:
            self.sync_now()
        if self.ready_log:
            if self.native is not None:  # leftovers launched by the native finalize
                n = len(self.ready_log)
                self.launch_log.extend((b, n) for b in range(len(self.launch_log), len(self.buckets)))
            self.ready_log_last, self.launch_log_last = list(self.ready_log), list(self.launch_log)
            self.maybe_rebuild()
        self.ready_log, self.launch_log = [], []

    def broadcast_params(self, module=None, src: int = 0):
        """DDP construction broadcast (distributed.py:864-870): one collective over the flat
        parameter buffer plus the module's buffers."""
        if not self.dp:
            return
        dist.broadcast(self.flat.param_buf, src=src, group=self.group)
        if module is not None:
            for b in module.buffers():
                dist.broadcast(b.data, src=src, group=self.group)

    def set_timing(self, on: bool = True):
        """Bracket the end-of-backward wait with GPU events: ``take_exposed_ms()`` then returns, per synchronised
        backward, the ms between the last backward kernel and the last bucket's all-reduce completing on the compute
        stream (communication not hidden under backward)."""
        self.timing = bool(on)
        if self.native is not None:
            self.native.set_timing(self.timing)

    def take_exposed_ms(self) -> list[float]:
        if self.native is not None:
            return list(self.native.take_exposed_ms())
        out, self._host_ms = list(self._host_ms), []
        for e0, e1 in self._events:
            e1.synchronize()
            out.append(e0.elapsed_time(e1))
        self._events.clear()
        return out

    def describe(self) -> dict:
        """The communication design this job runs (the entry points log it as their first JSON line): bucket size and
        how it was chosen, bucket count, overlap, wire dtype, engine."""
        return {"world_size": self.world, "backend": self.backend, "bucket_mb": self.bucket_mb,
                "bucket_choice": self.bucket_choice if self.bucket_choice is not None else "fixed",
                "n_buckets": len(self.buckets), "overlap": self.overlap,
                "wire_dtype": "bf16" if self.wire_dtype == torch.bfloat16 else str(self.flat.grad_buf.dtype).split(".")[-1],
                "engine": "native" if self.native is not None else "python"}

    def layout_signature(self) -> list[int]:
        """Bucket bounds + segment sizes: must be identical on every rank (RCCL matches collectives by order and
        size; a mismatch deadlocks or silently mixes gradients)."""
        sig = [len(self.buckets)] + [x for se in self.buckets for x in se]
        sig += [s.numel for s in self.flat.segments]
        return sig

    def launch_summary(self) -> dict:
        """The last synchronised backward's launch timeline: for each bucket (launch order) the fraction of gradient
        segments that were ready when it launched.  Overlap works when early buckets launch at small fractions."""
        n = max(1, len(self.flat.segments))
        log = self.launch_log_last
        fr = [round(k / n, 3) for _, k in log]
        return {"order": [b for b, _ in log], "ready_frac_at_launch": fr,
                "launched_before_backward_end": sum(1 for x in fr if x < 1.0), "n_buckets": len(self.buckets)}

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
