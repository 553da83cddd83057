"""Whole training step in one HIP graph (static shapes, one rank).

A step of the flagship model launches ~1,000 kernels; at the reference's small micro-batches (batch 1-8 per GPU,
ref/train-accelerator.py:169, ref/train-task.py:180, ref/train-torchrun.py:119,126) their host launch cost, not the
GPU, sets the step time.  ``GraphedStep`` captures forward + backward (+ the gradient-accumulation micro-steps) + the
global-norm clip + AdamW + zero_grad ONCE with ``torch.cuda.graph`` and then replays it: one host call per step.

What makes the replay a real training step and not a re-run of the captured one:

* dropout: the kernels mix a device step counter into every site seed (ops/rng.py StepSeed; the counter's ``add`` is
  inside the graph), and the host seed stream restarts every micro-step, so the seeds the graph baked in are the ones
  an eager step draws;
* AdamW reads [lr, lr / bc1, 1 / sqrt(bc2)] from a device tensor computed inside the graph from a device step count
  (ops/optim.py device_hyper), so the bias corrections advance; ``lr_fn(t)`` (device scalar -> device scalar) carries a
  schedule, default the optimizer's lr;
* inputs are copied into static buffers before each replay (same shapes required).

Not covered (eager instead): more than one rank (the gradient all-reduce is launched from autograd hooks with host-side
bucket bookkeeping), dynamic shapes, the Trainer's per-step host logic.  tests/test_graph_gpu.py checks graphed and
eager steps give the same parameters.
"""
from __future__ import annotations

import torch

from ..ops import rng as rng_mod


class GraphedStep:
    def __init__(self, engine, batches: list[dict], warmup: int = 2, lr_fn=None):
        if engine.reducer is not None:
            raise ValueError("GraphedStep: one rank only (the reducer's collectives are launched from autograd hooks)")
        if engine.env.device.type != "cuda":
            raise ValueError("GraphedStep: GPU only")
        self.eng = engine
        self.ga = len(batches)
        self.static = [{k: v.clone() for k, v in b.items() if torch.is_tensor(v)} for b in batches]
        engine.enable_step_seeds()
        opt = engine.optimizer
        dev = engine.env.device
        self.t = torch.full((), float(opt.step_count), dtype=torch.float32, device=dev)
        self.lr_fn = lr_fn
        self.loss = None
        # warmup on a side stream (lazy allocations, kernel attributes, GEMM solution lookups happen outside capture);
        # these are real training steps
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._body()
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = self._body()
        self._host_after_replay_sync()  # the capture ran the Python side once but executed nothing

    def _body(self):
        eng = self.eng
        total = None
        for k, b in enumerate(self.static):
            loss = eng.forward_backward(b, grad_accum=self.ga, sync=k == self.ga - 1)
            total = loss if total is None else total + loss
        self.t.add_(1.0)
        lr = self.lr_fn(self.t) if self.lr_fn is not None else eng.optimizer.param_groups[0]["lr"]
        eng.step(hyper=eng.optimizer.device_hyper(self.t, lr))
        return total / self.ga

    def _host_after_replay_sync(self):
        """Host mirrors of what a replay advances on the device (optimizer step count, dropout step counter) were
        advanced by the capture pass, which executed nothing: undo that."""
        eng = self.eng
        eng.optimizer.step_count -= 1
        eng.step_seed.host -= self.ga

    def replay(self, batches: list[dict] | None = None) -> torch.Tensor:
        """One training step on ``batches`` (copied into the static buffers; None: replay on the last ones).  Returns
        the mean loss of the step's micro-batches (device scalar, valid until the next replay)."""
        if batches is not None:
            if len(batches) != self.ga:
                raise ValueError(f"GraphedStep: {self.ga} micro-batches per step, got {len(batches)}")
            for st, b in zip(self.static, batches):
                for k, v in st.items():
                    v.copy_(b[k], non_blocking=True)
        self.graph.replay()
        self.eng.optimizer.step_count += 1
        self.eng.step_seed.host += self.ga
        rng_mod.default_rng().begin_micro_step()
        return self.loss
