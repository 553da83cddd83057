"""Accelerate-style facade over the native runtime (the API surface ref/train-accelerator.py uses).

``Accelerator()`` → process bootstrap (parallel/env.py; torchrun env → RCCL process group, or a single
process).  ``prepare(model, optimizer, train_dl, eval_dl)`` (accelerate/accelerator.py:1414):

* model → :class:`PreparedModel`: weights moved to the device in the compute dtype, parameters
  flattened, the bucketed RCCL reducer attached and parameters broadcast from rank 0 (what DDP's
  constructor does); calling it runs the fused-kernel model;
* a ``torch.optim.AdamW`` built on the raw model → :class:`~..ops.optim.FusedAdamW` over the flat
  buffers with the same lr / betas / eps and per-group weight decay (drop-in);
* a ``DataLoader`` → :class:`DeviceDataLoader` sharded like Accelerate's BatchSamplerShard
  (parallel/sampler.py) that moves batches to the device.

``backward`` (loss / GA + backward, reducer sync on the last micro-batch), ``gather``,
``pad_across_processes``, ``unwrap_model``, ``wait_for_everyone``, ``save_model``,
``clip_grad_norm_``, ``accumulate`` / ``no_sync`` complete the surface
(accelerator.py:2818, 3036, 3178, 3213, 3247).  Mixed precision defaults to bf16 on GPU (the
reference runs fp32; bf16 with fp32 master weights is this framework's documented default) and
fp32 on CPU.
"""
from __future__ import annotations

import contextlib

import torch

from ..ops.optim import FusedAdamW
from ..parallel import collectives
from ..parallel.env import init_distributed
from ..parallel.flat import FlatParams
from ..parallel.reducer import GradReducer, wire_dtype_of
from ..parallel.sampler import ShardedBatchSampler
from .engine import default_grad_dtype
from .schedule import LRScheduler


class PreparedModel(torch.nn.Module):
    def __init__(self, module, flat: FlatParams, reducer: GradReducer | None):
        super().__init__()
        self.module = module
        self.flat = flat
        self.reducer = reducer

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def generate(self, *args, **kwargs):
        return self.module.generate(*args, **kwargs)

    @property
    def config(self):
        return self.module.config

    def no_sync(self):
        return self.reducer.no_sync() if self.reducer is not None else contextlib.nullcontext()


class DeviceDataLoader:
    def __init__(self, dataset, batch_size, collate_fn, device, shuffle, num_replicas, rank, seed=0,
                 drop_last=False, even_batches=True, num_workers=0):
        self.dataset = dataset
        self.device = device
        self.batch_sampler = ShardedBatchSampler(len(dataset), batch_size, num_replicas, rank, shuffle, seed, drop_last,
                                                 even_batches)
        self.loader = torch.utils.data.DataLoader(dataset, batch_sampler=self.batch_sampler, collate_fn=collate_fn,
                                                  num_workers=num_workers,
                                                  pin_memory=device.type == "cuda")
        self.batch_size = batch_size

    def set_epoch(self, epoch):
        self.batch_sampler.set_epoch(epoch)

    def __len__(self):
        return len(self.batch_sampler)

    def __iter__(self):
        nb = self.device.type == "cuda"
        for batch in self.loader:
            yield {k: (v.to(self.device, non_blocking=nb) if torch.is_tensor(v) else v) for k, v in batch.items()}


class PreparedOptimizer:
    """Wraps FusedAdamW so it quacks like the torch optimizer the user built."""

    def __init__(self, opt: FusedAdamW, accelerator):
        self.opt = opt
        self.acc = accelerator
        self._clip = None

    @property
    def param_groups(self):
        return self.opt.param_groups

    def step(self):
        if self.acc.sync_gradients:
            self.opt.step(self._clip)
            self._clip = None

    def zero_grad(self, set_to_none: bool = False):
        if self.acc.sync_gradients:
            self.opt.zero_grad()

    def state_dict(self):
        return self.opt.state_dict()

    def load_state_dict(self, d):
        self.opt.load_state_dict(d)


class Accelerator:
    def __init__(self, mixed_precision: str | None = None, gradient_accumulation_steps: int = 1,
                 bucket_mb: float | str = "auto", overlap_comm: bool = True, cpu: bool = False, seed: int = 0,
                 even_batches: bool = True, grad_reduce_dtype: str | None = None):
        self.env = init_distributed(cpu=cpu if cpu else None)
        self.device = self.env.device
        if mixed_precision is None:
            mixed_precision = "bf16" if self.device.type == "cuda" else "no"
        self.mixed_precision = mixed_precision
        self.dtype = torch.bfloat16 if mixed_precision == "bf16" else torch.float32
        self.gradient_accumulation_steps = gradient_accumulation_steps
        self.bucket_mb = bucket_mb
        self.overlap_comm = overlap_comm
        self.grad_reduce_dtype = grad_reduce_dtype
        self.seed = seed
        self.even_batches = even_batches
        self.sync_gradients = True
        self._step = 0
        self._model: PreparedModel | None = None
        self._prepared_opts: list = []

    # ------------------------------------------------------------------ state
    @property
    def num_processes(self):
        return self.env.world_size

    @property
    def process_index(self):
        return self.env.rank

    @property
    def local_process_index(self):
        return self.env.local_rank

    @property
    def is_main_process(self):
        return self.env.is_main_process

    @property
    def is_local_main_process(self):
        return self.env.is_local_main_process

    @property
    def distributed_type(self):
        return "MULTI_GPU" if (self.env.world_size > 1 and self.device.type == "cuda") else \
            ("MULTI_CPU" if self.env.world_size > 1 else "NO")

    @property
    def state(self):
        return (f"Distributed environment: {self.distributed_type}  Backend: {self.env.backend}\n"
                f"Num processes: {self.num_processes}\nProcess index: {self.process_index}\n"
                f"Local process index: {self.local_process_index}\nDevice: {self.device}\n"
                f"Mixed precision type: {self.mixed_precision}\n")

    def print(self, *a, **kw):
        if self.is_local_main_process:
            print(*a, **kw)

    # ------------------------------------------------------------------ prepare
    def prepare(self, *objs):
        out = []
        # models first so optimizers can map their params onto the flat buffers
        order = sorted(range(len(objs)), key=lambda i: 0 if isinstance(objs[i], torch.nn.Module) else 1)
        res = [None] * len(objs)
        for i in order:
            res[i] = self._prepare_one(objs[i])
        out = res
        return out[0] if len(out) == 1 else tuple(out)

    def _prepare_one(self, obj):
        if isinstance(obj, PreparedModel):
            return obj
        if isinstance(obj, torch.nn.Module):
            return self.prepare_model(obj)
        if isinstance(obj, torch.optim.Optimizer):
            return self.prepare_optimizer(obj)
        if isinstance(obj, torch.utils.data.DataLoader):
            return self.prepare_data_loader(obj)
        return obj

    def prepare_model(self, model):
        model = model.to(device=self.device, dtype=self.dtype)
        flat = FlatParams(model, grad_dtype=default_grad_dtype(self.dtype))  # fp32 gradients (train/engine.py)
        reducer = None
        if self.env.world_size > 1:
            reducer = GradReducer(flat, bucket_mb=self.bucket_mb, overlap=self.overlap_comm,
                                  wire_dtype=wire_dtype_of(self.grad_reduce_dtype))
            reducer.broadcast_params(model)
        self._model = PreparedModel(model, flat, reducer)
        return self._model

    def prepare_optimizer(self, opt):
        if self._model is None:
            raise RuntimeError("prepare the model before (or together with) the optimizer")
        flat = self._model.flat
        g0 = opt.param_groups[0]
        decay_of = {}
        for g in opt.param_groups:
            for p in g["params"]:
                decay_of[id(p)] = g.get("weight_decay", 0.0)
        names = {id(p): s.name for s, p in zip(flat.segments, flat.params)}
        wds = {decay_of.get(id(p), 0.0) for p in flat.params}
        wd = max(wds) if wds else 0.0
        no_decay_names = {names[id(p)] for p in flat.params if decay_of.get(id(p), 0.0) == 0.0}
        fused = FusedAdamW(flat, lr=g0["lr"], betas=g0.get("betas", (0.9, 0.999)), eps=g0.get("eps", 1e-8),
                           weight_decay=wd, no_decay=(lambda n: n in no_decay_names) if wd else None)
        po = PreparedOptimizer(fused, self)
        self._prepared_opts.append(po)
        return po

    def prepare_data_loader(self, dl):
        shuffle = isinstance(dl.sampler, torch.utils.data.RandomSampler)
        bs = dl.batch_size if dl.batch_size is not None else 1
        return DeviceDataLoader(dl.dataset, bs, dl.collate_fn, self.device, shuffle, self.num_processes,
                                self.process_index, seed=self.seed, drop_last=dl.drop_last,
                                even_batches=self.even_batches, num_workers=dl.num_workers)

    # ------------------------------------------------------------------ training
    def backward(self, loss):
        ga = self.gradient_accumulation_steps
        m = self._model
        ctx = m.no_sync() if (m is not None and not self.sync_gradients) else contextlib.nullcontext()
        with ctx:
            (loss / ga if ga > 1 else loss).backward()
        if m is not None and m.reducer is not None and self.sync_gradients:
            m.reducer.post_backward()

    @contextlib.contextmanager
    def accumulate(self, model=None):
        self._step += 1
        self.sync_gradients = (self._step % self.gradient_accumulation_steps) == 0
        try:
            yield
        finally:
            pass

    def no_sync(self, model=None):
        m = model if isinstance(model, PreparedModel) else self._model
        return m.no_sync() if m is not None else contextlib.nullcontext()

    def make_train_step(self, model, optimizer, graph: bool | None = None):
        """The reference loop's per-batch body — ``outputs = model(**batch); accelerator.backward(outputs.loss);
        optimizer.step(); optimizer.zero_grad()`` (ref/train-accelerator.py:219-228) — as one callable
        ``step(batch) -> loss``, run by train/graph.py's StepRunner: replayed from a HIP graph once the batch shape
        repeats (GPU, unless ``graph=False`` / ``DLLM_GRAPH=0``), eager otherwise.  Gradient accumulation keeps the
        explicit loop (``accumulate`` / ``backward``).  ``clip_grad_norm_`` keeps its eager meaning: it applies to the
        next step only (call it every iteration to clip every step); a captured graph holds the clip it was captured
        with, so a step whose clip differs drops the graph and the runner captures again (StepRunner.invalidate)."""
        from .engine import TrainEngine
        from .graph import StepRunner
        m = model if isinstance(model, PreparedModel) else self._model
        po = optimizer if isinstance(optimizer, PreparedOptimizer) else self._prepared_opts[-1]
        if self.gradient_accumulation_steps != 1:
            raise ValueError("make_train_step: one micro-batch per optimizer step (use accumulate() for GA)")
        eng = TrainEngine.from_parts(m.module, self.env, m.flat, m.reducer, po.opt, max_grad_norm=None)
        runner = StepRunner(eng, enabled=graph)

        def step(batch: dict) -> torch.Tensor:
            clip, po._clip = po._clip, None  # requested for this step only (eager PreparedOptimizer.step semantics)
            if clip != eng.max_grad_norm:
                eng.max_grad_norm = clip
                runner.invalidate()
            self._step += 1
            self.sync_gradients = True
            losses, _ = runner([batch])
            return losses[0]

        step.runner = runner
        return step

    def clip_grad_norm_(self, parameters=None, max_norm: float = 1.0):
        """Clipping is fused into the next optimizer step (norm over the flat gradient buffer)."""
        for o in self._optimizers():
            o._clip = max_norm
        return None

    def _optimizers(self):
        return list(self._prepared_opts)

    # ------------------------------------------------------------------ collectives / utils
    def gather(self, t):
        if isinstance(t, dict):
            return {k: self.gather(v) for k, v in t.items()}
        if not torch.is_tensor(t):
            t = torch.tensor(t, device=self.device)
        return collectives.gather(t.to(self.device))

    def pad_across_processes(self, t, dim=0, pad_index=0, pad_first=False):
        return collectives.pad_across_processes(t, dim=dim, pad_index=pad_index, pad_first=pad_first)

    def reduce_mean(self, values: dict) -> dict:
        return collectives.mean_across_processes(values, self.device)

    def wait_for_everyone(self):
        collectives.barrier(device=self.device)

    def unwrap_model(self, model):
        return model.module if isinstance(model, PreparedModel) else model

    def save_model(self, model, output_dir, tokenizer=None):
        from ..platform.valohai import save_valohai_metadata
        return save_valohai_metadata(self.unwrap_model(model), output_dir, self.is_main_process, tokenizer)


def get_scheduler(name, optimizer, num_warmup_steps=0, num_training_steps=1):
    """transformers.get_scheduler equivalent for our optimizers (also accepts PreparedOptimizer)."""
    return LRScheduler(optimizer, name, num_warmup_steps, num_training_steps)
