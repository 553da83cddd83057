"""Whole training step replayed from HIP graphs (static shapes), one rank or data parallel.

A step of the flagship model launches ~1,000 kernels; at the reference's small micro-batches (batch 1-8 per GPU,
ref/train-accelerator.py:169, ref/train-task.py:180, ref/train-torchrun.py:119,126) their host launch cost, not the
GPU, sets the step time.  ``GraphedStep`` captures forward + backward (+ the gradient-accumulation micro-steps) + the
global-norm clip + AdamW + zero_grad with ``torch.cuda.graph`` and then replays it: one or two host calls per step.

Data parallel (an engine with a gradient reducer, parallel/reducer.py) is graphed in one of three schedules
(``comm``; default ops/routing.py ``graph_comm``, else "overlap" when the reducer overlaps, "split" with ``--no-overlap``):

* ``"overlap"`` (default): the forward + backward is captured as a CHAIN of graph segments cut at the reducer's bucket
  boundaries.  During the capture of the synchronised pass the reducer counts gradient readiness exactly as in an
  eager step but launches nothing (``GradReducer.begin_capture_cuts``); each time the next bucket(s) in bucket order
  become ready, the capture ends the current segment and begins the next one (same stream, same memory pool, relaxed
  capture mode: the cut runs on autograd's device thread).  A replay runs segment k, launches the buckets that became
  ready at the end of segment k as async RCCL all-reduces (their stream waits on the compute stream, so they run
  beside segment k+1), ..., then the compute stream waits on every bucket and the optimizer graph runs.  Same
  collective sequence as the eager engine, the overlap of the eager engine, and nothing of RCCL inside a graph.
  The bucket layout is the one rebuilt in gradient-ready order by the eager warm-up steps (rank 0's, broadcast), so
  every rank cuts at the same buckets; one host call per segment (≈8 at t5-base).
* ``"split"``: graph 1 = every micro-batch's forward + backward with the reducer disabled (gradients
  accumulate locally, like ``no_sync``); then the gradient all-reduce is issued EAGERLY between the replays — the
  reducer's launch schedule frozen to its bucket list (``GradReducer.sync_buckets``: the same buckets, in the same
  order, on every rank, each an async RCCL all-reduce; the compute stream waits on them without a host sync);
  graph 2 = clip + AdamW + zero_grad.  Nothing about RCCL is captured, so this is exactly the collective sequence
  the eager engine runs; what it gives up is the overlap of the all-reduce with backward (≈1 % of a t5-base step
  at per-GPU batch 512 over 8 GPUs, SURVEY.md §2.6 / bench.py ``comm``).
* ``"capture"``: ONE graph for the whole step; the reducer's bucket all-reduces are launched from the autograd
  hooks during capture, so RCCL's kernels are recorded into the graph at the point in backward where each bucket
  became ready (overlap preserved).  This needs RCCL's graph-capture support and a process group that tolerates
  capture (no async error handling); it is opt-in and covered by a 1-rank RCCL GPU test only.

What makes the replay a real training step and not a re-run of the captured one:

* dropout: the kernels mix a device step counter into every site seed (ops/rng.py StepSeed; the counter's ``add`` is
  inside the graph), and the host seed stream restarts every micro-step, so the seeds the graph baked in are the ones
  an eager step draws;
* AdamW reads [lr, lr / bc1, 1 / sqrt(bc2)] from a device tensor computed inside the graph from a device step count
  (ops/optim.py device_hyper), so the bias corrections advance; the learning rate is a device scalar refreshed from
  ``optimizer.param_groups[0]["lr"]`` before every replay (a scheduler or ``eng.step(lr=...)`` keeps working), or
  ``lr_fn(t)`` (device scalar -> device scalar) computes it inside the graph;
* inputs are copied into static buffers before each replay (same shapes required).

``use_graph=False`` runs the very same phase schedule eagerly (CPU / gloo tests of the schedule).

:class:`StepRunner` is how the entry points use it (train/trainer.py, train/accelerator.py ``make_train_step``,
train-task.py): the first steps of every new batch shape run eagerly (they are real training steps and warm up the
lazy state a capture must not see), the next step with the same shapes is captured and replayed, and any step whose
shapes differ (an epoch's last partial batch, dynamic padding) runs eagerly — the reference's max_length padding
(ref/train-accelerator.py:114-133) makes every full batch the same shape.  tests/test_graph_gpu.py checks graphed and
eager steps give the same parameters; tests/test_distributed_cpu.py checks the split schedule on 2 gloo ranks.
"""
from __future__ import annotations

import os

import torch

from ..ops import rng as rng_mod
from ..ops import routing

COMM_MODES = ("overlap", "split", "capture")


class GraphedStep:
    def __init__(self, engine, batches: list[dict], warmup: int = 2, lr_fn=None, comm: str | None = None,
                 use_graph: bool = True, num_items: bool = False, dp_ranks: int | None = None):
        """``batches``: the step's micro-batches (passes), whose shapes the graph fixes; ``warmup`` eager steps on them
        first (0: the caller already ran real steps of these shapes, StepRunner).  ``num_items``: the step's loss is
        normalised by a global token count handed to every ``replay`` (engine.forward_backward ``num_items`` /
        ``dp_ranks``, the Trainer's HF ``num_items_in_batch`` semantics); otherwise by the number of micro-batches."""
        dev = engine.env.device
        if use_graph and dev.type != "cuda":
            raise ValueError("GraphedStep: GPU only (use_graph=False runs the same schedule eagerly)")
        self.eng = engine
        self.red = engine.reducer
        default = "overlap" if (self.red is not None and self.red.overlap and self.red.dp) else "split"
        self.comm = (comm or routing.get("graph_comm") or default) if self.red is not None else None
        if self.comm == "overlap" and not (self.red.overlap and self.red.dp):
            self.comm = "split"  # no readiness hooks (--no-overlap) or nothing to reduce: post-backward buckets
        if self.comm is not None and self.comm not in COMM_MODES:
            raise ValueError(f"GraphedStep: comm must be one of {COMM_MODES}, got {self.comm!r}")
        self.use_graph = use_graph
        self.ga = len(batches)
        self.static = [{k: v.clone() for k, v in b.items() if torch.is_tensor(v)} for b in batches]
        engine.enable_step_seeds()
        opt = engine.optimizer
        self.t = torch.full((), float(opt.step_count), dtype=torch.float32, device=dev)
        self._t_host = opt.step_count  # what self.t holds (eager steps between replays move the optimizer's count)
        self.num_items = torch.ones((), dtype=torch.int64, device=dev) if num_items else None
        self.dp_ranks = dp_ranks
        self.losses: list = []  # per-pass mean losses of the last step (static outputs of the graph)
        self.lr_fn = lr_fn
        self._lr_host = float(opt.param_groups[0]["lr"])
        self.lr_t = torch.full((), self._lr_host, dtype=torch.float32, device=dev)
        self.loss = None
        self.norm = None
        if not use_graph:
            return
        # warmup on a side stream (lazy allocations, kernel attributes, GEMM solution lookups happen outside capture);
        # these are real training steps
        if warmup > 0:
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    self._eager_step()
            torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        self.t.fill_(float(opt.step_count))
        self._t_host = opt.step_count
        torch.cuda.empty_cache()  # eager blocks cached by the warmup are not usable by the graph's private pool
        _retire_collectives(self.red)
        # thread-local capture mode: only the capturing thread is barred from capture-unsafe HIP calls.  With the
        # default ("global") an unrelated thread's call during capture invalidates it — ProcessGroupNCCL's watchdog
        # thread polls the events of the warmup's all-reduces and aborts the process on that error (seen on a 1-rank
        # RCCL group).  Backward kernels launched from autograd's device thread onto the capture stream are captured
        # either way (capture is a property of the stream).
        mode = "thread_local"
        if self.comm == "overlap":
            self._capture_overlap()
        elif self.comm == "split":
            self.g_fb = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_fb, capture_error_mode=mode):
                self.loss = self._fb(sync=False)
            self.g_opt = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_opt, capture_error_mode=mode):
                self.norm = self._opt()
        else:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, capture_error_mode=mode):
                self.loss = self._fb(sync=True)
                self.norm = self._opt()
        self._host_after_capture()  # the capture ran the Python side once but executed nothing

    def _capture_overlap(self):
        """Segmented capture of forward + backward (module docstring, "overlap"), then the optimizer graph, all in one
        private memory pool (the graphs are replayed in the order they were captured)."""
        dev = self.eng.env.device
        red = self.red
        if red._rebuild_pending:
            raise RuntimeError("GraphedStep(overlap): the bucket layout must be rebuilt by an eager synchronised step "
                               "before capture (warmup >= 1 or a StepRunner eager step)")
        self._tick = torch.zeros(1, device=dev)  # one tiny kernel per cut: no segment is ever an empty graph
        self._pool = torch.cuda.graph_pool_handle()
        self._cap_stream = torch.cuda.Stream(dev)
        self.segments: list = []  # (graph, launch buckets up to this index after it, or None)
        import gc
        gc.collect()
        self._cap_stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self._cap_stream):
            self._seg = torch.cuda.CUDAGraph()
            self._seg.capture_begin(pool=self._pool, capture_error_mode="relaxed")
            red.begin_capture_cuts(self._cut)
            try:
                self.loss = self._fb(sync=True)
            finally:
                self.tail_buckets = red.end_capture_cuts()
                self._seg.capture_end()
            self.segments.append((self._seg, None))
            self._seg = None
            self.g_opt = torch.cuda.CUDAGraph()
            self.g_opt.capture_begin(pool=self._pool, capture_error_mode="relaxed")
            self.norm = self._opt()
            self.g_opt.capture_end()
        torch.cuda.current_stream(dev).wait_stream(self._cap_stream)

    def schedule(self) -> dict:
        """The data-parallel launch schedule a replay runs (bench.py ``comm``): for "overlap", the buckets launched
        between backward segments (before the backward ends) and the tail launched after it."""
        if self.comm != "overlap" or not self.use_graph:
            return {"schedule": self.comm}
        ups = [u for _, u in self.segments if u is not None]
        return {"schedule": "overlap", "segments": len(self.segments), "buckets_launched_before_backward_end":
                max(ups, default=0), "tail_buckets": list(self.tail_buckets), "n_buckets": len(self.red.buckets)}

    def _cut(self, buckets: list[int]):
        """Reducer callback during the segmented capture (autograd thread): buckets ``buckets`` just became ready —
        end the current segment here; the replay launches them after it."""
        from ..ops import streams
        with torch.cuda.stream(self._cap_stream):
            streams.join()  # side-stream gradient work (if any) belongs to this segment
            self._tick.add_(1.0)
            self._seg.capture_end()
            self.segments.append((self._seg, buckets[-1] + 1))
            self._seg = torch.cuda.CUDAGraph()
            self._seg.capture_begin(pool=self._pool, capture_error_mode="relaxed")

    # ------------------------------------------------------------------------------------------ phases
    def _fb(self, sync: bool):
        """Forward + backward of every micro-batch; ``sync``: the last one synchronises through the reducer hooks."""
        eng = self.eng
        total = None
        self.losses = []
        for k, b in enumerate(self.static):
            loss = eng.forward_backward(b, grad_accum=self.ga, sync=sync and k == self.ga - 1,
                                        num_items=self.num_items, dp_ranks=self.dp_ranks)
            self.losses.append(loss)
            total = loss if total is None else total + loss
        return total / self.ga

    def _comm(self):
        """Split mode, between the replays: the frozen bucket schedule, eagerly (no host sync on RCCL; with the
        reducer's timing on, its exposed-communication events bracket it)."""
        self.red.sync_buckets()

    def _opt(self):
        eng = self.eng
        self.t.add_(1.0)
        lr = self.lr_fn(self.t) if self.lr_fn is not None else self.lr_t
        return eng.step(hyper=eng.optimizer.device_hyper(self.t, lr))

    def _eager_step(self):
        """The step the graphs hold, run eagerly (warmup, and the use_graph=False schedule).  "overlap": the eager
        hook-launched reducer for the warm-up steps (they rebuild the buckets in ready order); with use_graph=False the
        segmented schedule itself — readiness counted in capture-cut mode, each cut launching its buckets at once."""
        if self.comm == "overlap" and not self.use_graph and not self.red._rebuild_pending:
            red = self.red
            red.begin_capture_cuts(lambda bs: red.launch_upto(bs[-1] + 1))
            try:
                loss = self._fb(sync=True)
            finally:
                red.end_capture_cuts()
            red.sync_buckets()
            return loss, self._opt()
        if self.comm == "split":
            loss = self._fb(sync=False)
            self._comm()
        else:
            loss = self._fb(sync=True)
        norm = self._opt()
        return loss, norm

    def _host_after_capture(self):
        """Host mirrors of what a replay advances on the device (optimizer step count, dropout step counter) were
        advanced by the capture pass, which executed nothing: undo that."""
        eng = self.eng
        eng.optimizer.step_count -= 1
        self._t_host = eng.optimizer.step_count
        eng.step_seed.host -= self.ga

    # ------------------------------------------------------------------------------------------ API
    def signature(self) -> tuple:
        return batch_signature(self.static)

    def replay(self, batches: list[dict] | None = None, num_items: torch.Tensor | None = None) -> torch.Tensor:
        """One training step on ``batches`` (copied into the static buffers; None: replay on the last ones).  Returns
        the mean loss of the step's micro-batches (device scalar, valid until the next replay; per pass: ``losses``)."""
        if batches is not None:
            if len(batches) != self.ga:
                raise ValueError(f"GraphedStep: {self.ga} micro-batches per step, got {len(batches)}")
            for st, b in zip(self.static, batches):
                for k, v in st.items():
                    v.copy_(b[k], non_blocking=True)
        if self.num_items is not None:
            if num_items is None:
                raise ValueError("GraphedStep: built with num_items=True, replay needs the step's token count")
            self.num_items.copy_(num_items, non_blocking=True)
        opt = self.eng.optimizer
        if opt.step_count != self._t_host:  # eager steps ran since the last replay: re-sync the bias corrections
            self.t.fill_(float(opt.step_count))
            self._t_host = opt.step_count
        lr = float(self.eng.optimizer.param_groups[0]["lr"])
        if lr != self._lr_host:
            self.lr_t.fill_(lr)
            self._lr_host = lr
        if not self.use_graph:
            self.loss, self.norm = self._eager_step()
            return self.loss
        if self.comm == "overlap":
            for g, upto in self.segments:
                g.replay()
                if upto is not None:
                    self.red.launch_upto(upto)
            self.red.sync_buckets()  # the tail buckets; the compute stream waits on every bucket (no host sync)
            self.g_opt.replay()
        elif self.comm == "split":
            self.g_fb.replay()
            self._comm()
            self.g_opt.replay()
        else:
            self.graph.replay()
        opt.step_count += 1
        self._t_host = opt.step_count
        self.eng.step_seed.host += self.ga
        rng_mod.default_rng().begin_micro_step()
        return self.loss


def batch_signature(batches: list[dict]) -> tuple:
    """What a captured graph fixes about a step's inputs: per pass, every tensor's name, shape and dtype."""
    return tuple(tuple(sorted((k, tuple(v.shape), v.dtype) for k, v in b.items() if torch.is_tensor(v)))
                 for b in batches)


def graphs_enabled(device: torch.device) -> bool:
    """Entry points replay their steps from HIP graphs on GPU unless ``DLLM_GRAPH=0``."""
    return device.type == "cuda" and os.environ.get("DLLM_GRAPH", "auto") != "0"


def graph_policy() -> str:
    """``DLLM_GRAPH``: ``auto`` (default) = capture, then keep the graph only if its replays are not slower than the
    eager steps of the same shape (StepRunner's timed probe); ``1`` = always replay; ``0`` = never capture."""
    v = os.environ.get("DLLM_GRAPH", "auto")
    return {"0": "off", "1": "on"}.get(v, "auto")


def _sig_key(sig) -> int:
    """A process-independent 62-bit key of a batch signature (Python's hash() of strings is salted per process)."""
    import hashlib
    return int.from_bytes(hashlib.sha256(repr(sig).encode()).digest()[:8], "little") >> 2


def _ranks_agree(sig, eng) -> bool:
    """Every rank of the default process group runs a step of signature ``sig`` (one tiny all-reduce; itself when
    there is no group).  The runner's capture and probe decisions issue collectives of their own, so they may only be
    taken on steps all ranks share."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() <= 1:
        return True
    dev = eng.env.device if dist.get_backend() == "nccl" else torch.device("cpu")
    k = _sig_key(sig)
    t = torch.tensor([k, -k], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t[0].item()) == -int(t[1].item())


def _retire_collectives(red) -> None:
    """Before a capture on an RCCL group: let ProcessGroupNCCL's watchdog retire every collective issued so far.  The
    watchdog thread polls the end events of the works it holds (every ~100 ms) until they complete; a poll landing
    inside a capture aborted the process once in the round-6 GPU suite (1-rank RCCL group, overlap schedule: the
    aborting thread had no Python frame, the autograd thread was mid-capture).  The device is synchronised, so the
    works are complete; two watchdog periods remove them from its list, and nothing is polled while capturing."""
    if red is None or not getattr(red, "dp", False):
        return
    import time
    import torch.distributed as dist
    try:
        backend = dist.get_backend(red.group)
    except Exception:  # noqa: BLE001 - no default group (single process): nothing to retire
        return
    if backend == "nccl":
        torch.cuda.synchronize()
        time.sleep(0.25)


def _all_ranks(flag: bool, eng) -> bool:
    """``flag`` AND-ed over the ranks of the default process group (itself when there is none)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() <= 1:
        return bool(flag)
    dev = eng.env.device if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


class StepRunner:
    """One optimizer step of an entry point's loop — forward + backward of the step's passes, gradient sync, clip +
    AdamW — eager or replayed from a HIP graph (GraphedStep).

    Per batch-shape signature: the first ``warmup`` steps run eagerly (real training steps; step seeds are on from
    the first one, so eager and replayed steps draw dropout masks from one stream), the next one is captured and from
    then on every step of that signature is a replay; steps of any other signature run eagerly.  ``enabled=False``
    (CPU, ``DLLM_GRAPH=0``) is the plain eager step.

    Policy ``auto`` (default, graph_policy): the last eager warm-up steps and the first ``PROBE`` replays of a signature
    are timed with device events (no host synchronisation until the decision); if the replays' median is slower than
    the eager steps' median by more than ``GRAPH_TOL``, the graph is dropped and the signature stays eager (at large
    micro-batches launch overhead is nil and a replay can lose to the eager stream; at small ones the graph wins by
    tens of percent).  The outcome is ``decision`` (logged by the entry points)."""

    PROBE = 3
    GRAPH_TOL = 0.003

    def __init__(self, engine, enabled: bool | None = None, warmup: int = 2, num_items: bool = False,
                 dp_ranks: int | None = None, comm: str | None = None):
        self.eng = engine
        self.enabled = graphs_enabled(engine.env.device) if enabled is None else bool(enabled)
        self.warmup = max(1, int(warmup))
        self.num_items = num_items
        self.dp_ranks = dp_ranks
        self.comm = comm
        self.graph: GraphedStep | None = None
        self.graph_error: str | None = None
        self._sig = None
        self._seen = 0
        self.replays = 0
        self.eager_steps = 0
        # the timed probe needs device events: on the CPU schedule (tests) an enabled runner always replays
        self.policy = ("off" if not self.enabled else graph_policy() if engine.env.device.type == "cuda" else "on")
        if self.policy == "auto":  # the probe's eager baseline: PROBE timed eager steps after the untimed first one
            self.warmup = max(self.warmup, 1 + self.PROBE)
        self.decision: dict | None = None  # auto policy: {"graph": bool, "eager_ms": .., "replay_ms": ..}
        self._eager_t: list = []   # (start, end) events of this signature's eager steps
        self._replay_t: list = []  # ... and of its first replays
        self._eager_sigs: set = set()  # signatures the probe sent back to eager steps
        if self.enabled:
            engine.enable_step_seeds()
        # multi-rank runs: a step that does not finish within DLLM_STEP_TIMEOUT ends the rank with a report of where it
        # stood (utils/watchdog.py); single-process runs have no partner to wait for
        self.watchdog = None
        self.steps = 0
        if engine.reducer is not None and engine.reducer.dp:
            from ..utils.watchdog import StepWatchdog
            wd = StepWatchdog(engine.env.rank, describe=self._where)
            self.watchdog = wd if wd.enabled else None

    def _where(self) -> dict:
        red = self.eng.reducer
        out = {"graph": self.graph is not None, "replays": self.replays, "eager_steps": self.eager_steps}
        if red is not None:
            out.update(n_buckets=len(red.buckets), buckets_launched=red._launched_count(),
                       bucket_bounds=[list(b) for b in red.buckets[:4]] + (["..."] if len(red.buckets) > 4 else []))
        return out

    def comm_report(self) -> dict:
        """The communication design this runner's steps use (entry points: first JSON line): the reducer's bucket
        choice and layout (GradReducer.describe) plus the graph policy and the data-parallel graph schedule."""
        red = self.eng.reducer
        rep = red.describe() if red is not None else {"world_size": self.eng.env.world_size, "reducer": None}
        if red is not None and red.dp:
            # every rank's bucket layout (RCCL pairs collectives by order and size): they must be identical
            import hashlib
            import json as _json
            import torch.distributed as dist
            sha = hashlib.sha1(_json.dumps(red.layout_signature()).encode()).hexdigest()[:16]
            shas = [None] * dist.get_world_size(red.group)
            dist.all_gather_object(shas, sha, group=red.group)
            if len(set(shas)) != 1:
                raise RuntimeError(f"gradient bucket layouts differ across ranks: {shas}")
            rep.update(bucket_layout_sha=sha, bucket_layouts_agree=True)
        sched = None
        if red is not None and self.policy != "off":
            default = "overlap" if (red.overlap and red.dp) else "split"
            sched = self.comm or routing.get("graph_comm") or default
            if sched == "overlap" and not (red.overlap and red.dp):
                sched = "split"
        rep.update(graph_policy=self.policy, graph_schedule=sched,
                   eager_schedule=("hook-overlap" if red is not None and red.overlap else "post-backward")
                   if red is not None else None,
                   step_timeout_s=self.watchdog.timeout_s if self.watchdog is not None else 0)
        return rep

    def invalidate(self):
        """Something a captured graph baked in changed (e.g. the clip norm): drop the graph; the next steps of the
        signature run eagerly again and are re-captured after ``warmup`` of them."""
        if self.graph is not None:
            torch.cuda.synchronize()
        self.graph = None
        self._sig = None
        self._seen = 0

    def __call__(self, passes: list[dict], num_items: torch.Tensor | None = None, lr: float | None = None):
        """Run one step; returns (per-pass mean losses, pre-clip grad norm or None) as device tensors."""
        wd = self.watchdog
        if wd is None:
            return self._step(passes, num_items, lr)
        self.steps += 1
        wd.begin(self.steps)
        try:
            return self._step(passes, num_items, lr)
        finally:
            wd.end(self.eng.env.device)

    def _step(self, passes, num_items, lr):
        eng = self.eng
        if lr is not None:
            eng.optimizer.param_groups[0]["lr"] = lr
        timed = None
        if self.enabled:
            sig = batch_signature(passes)
            g = self.graph
            # while the runner may still capture or probe, its decisions run collectives: take them only on steps whose
            # signature every rank shares (a disagreeing step runs eagerly and counts for nothing)
            unsettled = (g is None and self.graph_error is None and sig not in self._eager_sigs) or (
                g is not None and self.policy == "auto" and self.decision is None)
            if unsettled and not _ranks_agree(sig, eng):
                return self._eager(passes, num_items, None)
            if g is not None and sig == g.signature():
                probing = self.policy == "auto" and self.decision is None
                if probing and len(self._replay_t) >= self.PROBE:
                    self._decide()
                    if self.graph is None:
                        return self._step(passes, num_items, None)
                    probing = False
                ev = self._events() if probing else None
                g.replay(passes, num_items=num_items)
                if ev is not None:
                    ev[1].record()
                    self._replay_t.append(ev)
                self.replays += 1
                return list(g.losses), g.norm
            if g is None and self.graph_error is None and sig not in self._eager_sigs:
                self._seen = self._seen + 1 if sig == self._sig else 1
                self._sig = sig
                if self._seen > self.warmup:
                    # a failed capture executed nothing on the device, but its host pass may have advanced the host
                    # mirrors of device state: snapshot them
                    rng = rng_mod.default_rng()
                    snap = (eng.optimizer.step_count, eng.step_seed.host, rng.counter)
                    err = None
                    try:
                        self.graph = GraphedStep(eng, passes, warmup=0, comm=self.comm,
                                                 num_items=num_items is not None, dp_ranks=self.dp_ranks)
                    except Exception as e:  # noqa: BLE001 - capture unsupported here: stay eager, say why once
                        err = f"{type(e).__name__}: {str(e)[:300]}"
                    # every data-parallel rank must take the same schedule (graph replays vs eager steps issue their
                    # collectives differently): a capture failure anywhere sends all ranks back to eager steps
                    if not _all_ranks(err is None, eng):
                        err = err or "HIP graph capture failed on another rank"
                    if err is not None:
                        self.graph = None
                        eng.optimizer.step_count, eng.step_seed.host, rng.counter = snap
                        self.graph_error = err
                        from ..utils.logging import get_logger
                        get_logger(__name__).warning(f"HIP graph capture failed, eager steps: {self.graph_error}")
                        torch.cuda.synchronize()
                    else:
                        return self._step(passes, num_items, None)
            # the eager steps of the signature that will be captured are the probe's baseline (not the first one: it
            # carries the lazy initialisation)
            if self.policy == "auto" and self.decision is None and sig == self._sig and self._seen >= 2:
                timed = self._events()
        return self._eager(passes, num_items, timed)

    def _eager(self, passes, num_items, timed):
        eng = self.eng
        self.eager_steps += 1
        losses = []
        for j, pb in enumerate(passes):
            losses.append(eng.forward_backward(pb, grad_accum=len(passes), sync=j + 1 == len(passes),
                                               num_items=num_items, dp_ranks=self.dp_ranks))
        norm = eng.step()
        if timed is not None:
            timed[1].record()
            self._eager_t.append(timed)
        return losses, norm

    @staticmethod
    def _events():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        return e0, e1

    def _decide(self):
        """Auto policy: keep the graph iff its replays are not slower than the eager steps (medians)."""
        import statistics
        self._replay_t[-1][1].synchronize()
        med = lambda evs: statistics.median(a.elapsed_time(b) for a, b in evs)  # noqa: E731
        eager = med(self._eager_t[-self.PROBE:]) if self._eager_t else float("inf")
        replay = med(self._replay_t)
        # one decision for all data-parallel ranks (their schedules must match): graphs only if every rank keeps them
        keep = _all_ranks(replay <= eager * (1.0 + self.GRAPH_TOL), self.eng)
        self.decision = {"graph": keep, "eager_ms": round(eager, 3), "replay_ms": round(replay, 3)}
        if not keep:
            self._eager_sigs.add(self.graph.signature())
            self.graph = None
        self._eager_t, self._replay_t = [], []
