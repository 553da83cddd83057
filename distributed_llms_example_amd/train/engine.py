"""The training step every loop shares: model → flat params → gradient reducer → fused AdamW.

Both the Trainer-style loop (train/trainer.py, ref/train-torchrun.py) and the Accelerate-style
facade (train/accelerator.py, ref/train-accelerator.py / train-task.py) — and bench.py — dispatch to
this one engine and therefore to the same kernel library and the same RCCL reducer (BASELINE.json
north star: "both loops dispatch to the same kernel library").
"""
from __future__ import annotations

import contextlib
import os

import torch

from ..ops import gemm
from ..ops import rng as rng_mod
from ..ops import streams
from ..ops.optim import FusedAdamW
from ..utils import profiling
from ..parallel.env import DistEnv
from ..parallel.flat import FlatParams
from ..parallel.reducer import DEFAULT_BUCKET_MB, GradReducer, wire_dtype_of

# transformers Trainer.get_decay_parameter_names: no decay for biases and norm weights (trainer.py:1305-1315)
def default_no_decay(name: str) -> bool:
    n = name.lower()
    return n.endswith(".bias") or "layer_norm" in n or "layernorm" in n or "norm.weight" in n


def default_grad_dtype(param_dtype: torch.dtype) -> torch.dtype:
    """Gradient buffer dtype: fp32 (the reference's HF Trainer / Accelerate keep fp32 gradients, and GA sums
    16 micro-batches, ref/train-torchrun.py:126) unless ``DLLM_GRAD_DTYPE=bf16`` opts into param-dtype
    gradients (half the all-reduce bytes, every accumulation rounded to 8 mantissa bits)."""
    choice = os.environ.get("DLLM_GRAD_DTYPE", "fp32").lower()
    if choice in ("bf16", "param", "same"):
        return param_dtype
    return torch.float32


def token_count(labels: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Non-ignored target tokens of a micro-batch, as a device scalar (no host sync)."""
    return (labels != ignore_index).sum()


class TrainEngine:
    def __init__(self, model: torch.nn.Module, env: DistEnv, *, lr: float = 5e-5, weight_decay: float = 0.0,
                 betas=(0.9, 0.999), eps: float = 1e-8, max_grad_norm: float | None = 1.0,
                 dtype: torch.dtype = torch.bfloat16, bucket_mb: float | str = DEFAULT_BUCKET_MB, overlap: bool = True,
                 no_decay=default_no_decay, label_smoothing: float = 0.0, grad_dtype: torch.dtype | None = None,
                 force_reducer: bool = False, grad_reduce_dtype: str | None = None):
        """``bucket_mb``: MiB per all-reduce bucket, or "auto" (parallel/reducer.py choose_bucket_mb: probed on the
        job's process group, recorded in ``reducer.bucket_choice``).  ``grad_reduce_dtype``: "bf16" compresses each bucket
        for the wire only (fp32 accumulation kept), None / "fp32" reduces the gradient buffer as it is."""
        self.env = env
        self.model = model.to(device=env.device, dtype=dtype)
        self.dtype = dtype
        self.flat = FlatParams(self.model, grad_dtype=grad_dtype or default_grad_dtype(dtype))
        streams.tag_roles(self.model)  # layer roles for the paired side-stream policy (ops/streams.py)
        # force_reducer: a reducer (and its collectives) on a 1-rank process group — GPU tests of the RCCL paths
        self.reducer = (GradReducer(self.flat, bucket_mb=bucket_mb, overlap=overlap, force=force_reducer,
                                    wire_dtype=wire_dtype_of(grad_reduce_dtype))
                        if env.world_size > 1 or force_reducer else None)
        if self.reducer is not None:
            self.reducer.broadcast_params(self.model)
        self.optimizer = FusedAdamW(self.flat, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                    no_decay=no_decay)
        self.max_grad_norm = max_grad_norm
        self.label_smoothing = label_smoothing
        self.step_seed: rng_mod.StepSeed | None = None
        self._init_defer()

    # micro-batches of at most this many input tokens defer their weight gradients to the window's last one
    DEFER_MAX_TOKENS = 16384

    def _init_defer(self):
        """Deferred weight gradients for gradient accumulation (ops/gemm.py WgradDefer): ``DLLM_DEFER_WGRAD`` = auto
        (micro-batches of <= DEFER_MAX_TOKENS input tokens on the GPU), 1 (always), 0 (never).  Kept operands end the
        window's deferral early past 60 % of the device memory."""
        cap = None
        if self.env.device.type == "cuda":
            cap = int(0.6 * torch.cuda.get_device_properties(self.env.device).total_memory)
        self.wgrad_defer = gemm.WgradDefer(mem_cap=cap)
        self._defer_mode = os.environ.get("DLLM_DEFER_WGRAD", "auto").lower()
        self._ga_k = 0
        # callers that measure one micro-batch's activation memory (train/trainer.py coalescing) switch deferral off for
        # that step: the kept operands of the whole window would count as one micro-batch's activations
        self.defer_enabled = True

    def _defer_for(self, batch: dict, grad_accum: int) -> gemm.WgradDefer | None:
        if grad_accum <= 1 or not self.defer_enabled or self._defer_mode in ("0", "off", "false"):
            return None
        if self._defer_mode == "auto":
            ids = batch.get("input_ids")
            if self.env.device.type != "cuda" or ids is None or ids.numel() > self.DEFER_MAX_TOKENS:
                return None
        return self.wgrad_defer

    @classmethod
    def from_parts(cls, model: torch.nn.Module, env: DistEnv, flat: FlatParams, reducer: GradReducer | None,
                   optimizer: FusedAdamW, max_grad_norm: float | None = None, label_smoothing: float = 0.0):
        """An engine over state another front end already built (train/accelerator.py: the prepared model's flat
        buffers and reducer, the prepared optimizer), so its loop can run the same step — and the same HIP-graph
        step runner (train/graph.py) — as the Trainer."""
        eng = cls.__new__(cls)
        eng.env, eng.model, eng.dtype = env, model, flat.dtype
        eng.flat, eng.reducer, eng.optimizer = flat, reducer, optimizer
        eng.max_grad_norm, eng.label_smoothing = max_grad_norm, label_smoothing
        eng.step_seed = None
        eng._init_defer()
        return eng

    def enable_step_seeds(self, start: int | None = None) -> rng_mod.StepSeed:
        """Dropout seeds that a captured HIP graph can replay (ops/rng.py StepSeed): from now on every micro-step
        advances a device counter the kernels mix into each site seed, and the host seed stream restarts per micro-step.
        Masks differ from the default mode's (another, equally uniform, stream), so enable it before training."""
        if self.step_seed is None:
            self.step_seed = rng_mod.StepSeed(self.env.device)
            self.step_seed.enable()
        if start is not None:  # resumed run (train/checkpoint.py "step_seed")
            self.step_seed.t.fill_(int(start))
            self.step_seed.host = int(start)
        return self.step_seed

    def disable_step_seeds(self) -> None:
        """Back to the default dropout seed stream: the kernels' device step pointer, the active-step registry and the
        host stream's site mode are all restored (StepSeed.disable), and forward_backward stops advancing it."""
        if self.step_seed is not None:
            self.step_seed.disable()
            self.step_seed = None

    def no_sync(self):
        return self.reducer.no_sync() if self.reducer is not None else contextlib.nullcontext()

    def forward(self, batch: dict):
        self.flat.reset_pending()
        return self.model(input_ids=batch["input_ids"], attention_mask=batch.get("attention_mask"),
                          decoder_input_ids=batch.get("decoder_input_ids"), labels=batch["labels"],
                          label_smoothing=self.label_smoothing)

    def backward(self, loss: torch.Tensor, scale: float = 1.0, sync: bool = True):
        ctx = contextlib.nullcontext() if sync else self.no_sync()
        with ctx:
            (loss * scale if scale != 1.0 else loss).backward()
        if sync and self.reducer is not None:
            self.reducer.post_backward()

    def forward_backward(self, batch: dict, grad_accum: int = 1, sync: bool = True,
                         num_items: torch.Tensor | None = None, dp_ranks: int | None = None) -> torch.Tensor:
        """Forward + backward of one micro-batch; returns its mean loss (detached).

        ``num_items``: the GLOBAL number of non-ignored target tokens of the whole optimizer step (all GA
        micro-batches on all data-parallel ranks, a device scalar).  Given, the gradient is that of
        Σ token losses / num_items — every token weighs the same however the tokens are spread over
        micro-batches and ranks (HF Trainer ``num_items_in_batch``); the reducer's average
        over ranks is undone by the number of data-parallel ranks ``dp_ranks`` whose tokens ``num_items``
        counts (default: the reducer's world; context-parallel ranks share one batch and count once).  Without it each micro-batch mean is divided by
        ``grad_accum`` (identical when every micro-batch has the same token count)."""
        ctx = contextlib.nullcontext() if sync else self.no_sync()
        if self.step_seed is not None:
            self.step_seed.advance()
            rng_mod.default_rng().begin_micro_step()
        # weight gradients on a side stream (ops/streams.py) unless the reducer launches all-reduces from the hooks
        # of this backward (those order themselves after the compute stream only)
        hooks_reduce = self.reducer is not None and sync and self.reducer.overlap and self.reducer.dp
        ids = batch.get("input_ids")
        side = streams.scope(streams.default_enabled(ids.numel() if ids is not None else None) and not hooks_reduce
                             and self.env.device.type == "cuda")
        # the accumulation window ends at the synchronising micro-batch, or after grad_accum of them (a graph's split
        # schedule runs every micro-batch unsynchronised and reduces after the last)
        self._ga_k += 1
        last = sync or self._ga_k >= grad_accum
        if last:
            self._ga_k = 0
        dfr = self._defer_for(batch, grad_accum)
        if dfr is None and last and self.wgrad_defer.active and self.wgrad_defer.pending():
            # a last micro-batch that does not defer itself (too many tokens) still closes the window the earlier ones
            # opened: its weight-gradient GEMMs merge the kept segments in the backward, before the hooks that launch
            # the overlapped bucket all-reduces fire (a flush after backward() would add them after the reduction)
            dfr = self.wgrad_defer
        with ctx, side, gemm.defer_wgrads(dfr, final=last):
            with profiling.range("forward"):
                out = self.forward(batch)
                loss = out.loss
            with profiling.range("backward" if sync else "backward(no_sync)"):
                if num_items is not None:
                    w = dp_ranks if dp_ranks is not None else (self.reducer.world if self.reducer is not None else 1)
                    scale = token_count(batch["labels"]).to(torch.float32) * w / num_items.to(torch.float32)
                    (loss * scale).backward()
                else:
                    (loss / grad_accum if grad_accum > 1 else loss).backward()
        if last:
            # weights the last micro-batch did not touch, before the reducer's post-backward launches their buckets
            if self.wgrad_defer.pending():
                self.wgrad_defer.flush()
            self.wgrad_defer.active = True
        elif dfr is not None and dfr.mem_cap is not None and torch.cuda.memory_allocated(self.env.device) > dfr.mem_cap:
            dfr.flush()
            dfr.active = False  # the rest of this window runs undeferred
        if sync and self.reducer is not None:
            with profiling.range("allreduce(post_backward)"):
                self.reducer.post_backward()
        return loss.detach()

    def step(self, lr: float | None = None, hyper: torch.Tensor | None = None):
        """Clip + AdamW + zero_grad.  Returns the pre-clip grad norm as a device tensor (or None).  ``hyper``: device
        [lr, lr / bc1, 1 / sqrt(bc2)] (graph mode, ops/optim.py device_hyper)."""
        if lr is not None:
            self.optimizer.param_groups[0]["lr"] = lr
        if self.wgrad_defer.pending():  # a window left open (fewer micro-batches than its grad_accum)
            self.wgrad_defer.flush()
        self.wgrad_defer.active = True
        self._ga_k = 0
        with profiling.range("optimizer(clip+adamw)"):
            norm = self.optimizer.step(self.max_grad_norm, hyper=hyper)
            self.optimizer.zero_grad()
        return norm

    def train(self, mode: bool = True):
        self.model.train(mode)
        return self
