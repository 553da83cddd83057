"""Trainer-style loop (the HF Trainer path of ref/train-torchrun.py) on the native runtime.

Semantics kept from transformers' Trainer as the reference configures it:
``TrainingArguments`` names and defaults (lr 5e-5, betas (0.9, 0.999), eps 1e-8, max_grad_norm 1.0,
linear schedule with ``warmup_steps``, seed 42, weight decay excluded for biases / norm weights),
gradient accumulation with ``no_sync`` on all but the last micro-batch, clip → AdamW → scheduler →
zero_grad on the sync step, ``logging_steps`` JSON logs through callbacks (``loss`` = mean over the
logged micro-batches — the true mean, not the GA-summed value 5.15 prints, Appendix A Q12;
``grad_norm``, ``learning_rate``, ``epoch``), eval every ``eval_steps`` (eval loss; the reference's
eval set is passed untokenised and crashes, Q3 — here it is tokenised), checkpoints every
``save_steps`` and at the last step, final ``train_runtime`` / ``train_samples_per_second`` /
``train_steps_per_second`` / ``train_loss`` (trainer_utils.py:531-558).  Accepts both
``evaluation_strategy`` and ``eval_strategy`` and both ``tokenizer`` and ``processing_class`` (Q2).

The step itself is train/engine.py's: flat params, bucketed RCCL reducer, fused kernels, fused AdamW.
"""
from __future__ import annotations

import dataclasses
import math
import os
import time
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from ..ops.rng import manual_seed
from ..parallel import collectives
from ..parallel.context import shard_sequence
from ..parallel.env import init_distributed
from ..parallel.sampler import ShardedBatchSampler
from ..utils.logging import get_logger
from .callbacks import CallbackHandler, DefaultFlowCallback, TrainerControl, TrainerState
from ..utils import faults
from .checkpoint import latest_checkpoint, load_checkpoint, save_checkpoint
from .engine import TrainEngine, default_no_decay, token_count
from .graph import StepRunner, graphs_enabled
from .schedule import LRScheduler

logger = get_logger(__name__)


@dataclass
class TrainingArguments:
    output_dir: str = "output"
    num_train_epochs: float = 1.0
    max_steps: int = -1
    per_device_train_batch_size: int = 8
    per_device_eval_batch_size: int = 8
    gradient_accumulation_steps: int = 1
    learning_rate: float = 5e-5
    weight_decay: float = 0.0
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_epsilon: float = 1e-8
    max_grad_norm: float = 1.0
    lr_scheduler_type: str = "linear"
    warmup_steps: int = 0
    warmup_ratio: float = 0.0
    logging_steps: int = 500
    eval_strategy: str = "no"
    evaluation_strategy: str | None = None
    eval_steps: int | None = None
    save_strategy: str = "steps"
    save_steps: float = 500
    save_total_limit: int | None = None
    seed: int = 42
    label_smoothing_factor: float = 0.0
    bf16: bool | None = None
    dataloader_num_workers: int = 0
    dataloader_drop_last: bool = False
    ddp_find_unused_parameters: bool | None = None
    ddp_bucket_cap_mb: float | str | None = "auto"  # MiB, or "auto"/None (parallel/reducer.py choose_bucket_mb)
    ddp_timeout: int = 1800
    overlap_comm: bool = True
    grad_reduce_dtype: str = "fp32"  # "bf16": compress each gradient bucket for the wire (fp32 accumulation kept)
    context_parallel_size: int = 1  # shard the encoder sequence over groups of this many consecutive ranks
    resume_from_checkpoint: str | None = None
    nan_guard: bool = True  # raise when the (logged, already synchronised) mean loss is NaN/Inf
    # Run an optimizer step's gradient-accumulation micro-batches as fewer, larger forward/backward passes (same
    # samples, same token-count normalisation, same single optimizer step).  The reference accumulates 16 micro-batches
    # of 8 because its GPUs lack memory; a 288 GB MI355X holds the whole group, and one pass of 128 runs ~2x the
    # samples/s of 16 launch-bound passes of 8 (profiles/r2_entry_points.md).  "auto": as many micro-batches per pass
    # as the first step's measured activation memory allows within coalesce_memory_fraction of the device (GPU only);
    # an int caps the samples per pass (0 / 1: off).
    coalesce_grad_accum: str | int = "auto"
    coalesce_memory_fraction: float = 0.6
    report_to: list = field(default_factory=list)

    def __post_init__(self):
        if self.evaluation_strategy is not None:
            self.eval_strategy = self.evaluation_strategy
        if self.eval_strategy == "steps" and not self.eval_steps:
            self.eval_steps = self.logging_steps

    def to_dict(self):
        return dataclasses.asdict(self)


@dataclass
class TrainOutput:
    global_step: int
    training_loss: float
    metrics: dict


class Trainer:
    def __init__(self, model, args: TrainingArguments, train_dataset=None, eval_dataset=None, data_collator=None,
                 callbacks=None, tokenizer=None, processing_class=None, compute_metrics=None, env=None):
        self.args = args
        self.env = env or init_distributed(timeout_s=args.ddp_timeout)
        self.tokenizer = processing_class if processing_class is not None else tokenizer
        torch.manual_seed(args.seed)
        # context parallelism (parallel/context.py): ranks [k*cp, (k+1)*cp) share one batch and one dropout stream
        cp = max(1, int(args.context_parallel_size))
        assert self.env.world_size % cp == 0, "world size must be a multiple of context_parallel_size"
        self.dp_rank, self.dp_world = self.env.rank // cp, self.env.world_size // cp
        self.cp_group = None
        if cp > 1:
            for k in range(self.dp_world):  # every rank creates every group (c10d requirement)
                grp = dist.new_group(list(range(k * cp, (k + 1) * cp)))
                if k == self.dp_rank:
                    self.cp_group = grp
            model.enable_context_parallel(self.cp_group)
        manual_seed(args.seed + 7919 * self.dp_rank)
        bf16 = args.bf16 if args.bf16 is not None else self.env.device.type == "cuda"
        self.dtype = torch.bfloat16 if bf16 else torch.float32
        self.engine = TrainEngine(model, self.env, lr=args.learning_rate, weight_decay=args.weight_decay,
                                  betas=(args.adam_beta1, args.adam_beta2), eps=args.adam_epsilon,
                                  max_grad_norm=args.max_grad_norm, dtype=self.dtype,
                                  bucket_mb=args.ddp_bucket_cap_mb or "auto", overlap=args.overlap_comm,
                                  grad_reduce_dtype=args.grad_reduce_dtype,
                                  no_decay=default_no_decay, label_smoothing=args.label_smoothing_factor)
        self.model = self.engine.model
        self.train_dataset = train_dataset
        self.eval_dataset = eval_dataset
        self.data_collator = data_collator
        self.compute_metrics = compute_metrics
        self.handler = CallbackHandler([DefaultFlowCallback] + list(callbacks or []))
        self.state = TrainerState(is_world_process_zero=self.env.is_main_process)
        self.control = TrainerControl()
        self.scheduler = None

    # ------------------------------------------------------------------ data
    def _loader(self, dataset, batch_size, shuffle, epoch=0, cp=True):
        world, rank = (self.dp_world, self.dp_rank) if cp else (self.env.world_size, self.env.rank)
        sampler = ShardedBatchSampler(len(dataset), batch_size, world, rank, shuffle=shuffle,
                                      seed=self.args.seed, drop_last=self.args.dataloader_drop_last)
        sampler.set_epoch(epoch)
        return torch.utils.data.DataLoader(dataset, batch_sampler=sampler, collate_fn=self.data_collator,
                                           num_workers=self.args.dataloader_num_workers,
                                           pin_memory=self.env.device.type == "cuda"), sampler

    def _coalesce_cap(self) -> int | None:
        """Max padded tokens (samples x padded sequence lengths, _padded_tokens) per forward/backward pass when coalescing
        micro-batches; None = off, -1 = decide after step 1.  An explicit integer setting counts micro-batches of the
        configured batch size at the first group's padded lengths."""
        v = self.args.coalesce_grad_accum
        if self.cp_group is not None or self.args.gradient_accumulation_steps <= 1:
            return None
        if str(v) == "auto":
            return -1 if self.env.device.type == "cuda" else None
        v = int(v)
        return v if v > 1 else None

    @staticmethod
    def _padded_tokens(batches) -> int:
        """Tokens of ONE pass over ``batches`` after _merge pads every sequence dim to the group maximum: samples x
        (max source length + max target length).  The coalescing budget is counted in these, not in samples, so a
        later group of longer (dynamically padded) sequences cannot exceed the memory measured at step 1."""
        n = sum(b["labels"].shape[0] for b in batches)
        src = max((b["input_ids"].shape[1] for b in batches if "input_ids" in b), default=0)
        tgt = max(b["labels"].shape[1] for b in batches)
        return n * (src + tgt)

    def _auto_cap(self, base_bytes: int, peak_bytes: int, step1_tokens: int) -> int | None:
        """Padded-token budget per pass from the first step: peak - base = the activations of one micro-batch of the
        step's largest padded size (+ transient buffers).  Attention memory grows faster than linearly with sequence
        length (the S^2 score tiles are never materialised here, but the dropout bit planes are), so the budget keeps
        a margin below the memory fraction."""
        total = torch.cuda.get_device_properties(self.env.device).total_memory
        act = max(1, peak_bytes - base_bytes)
        k = int((self.args.coalesce_memory_fraction * total - base_bytes) // act)
        k = min(k, self.args.gradient_accumulation_steps)
        if self.dp_world > 1:  # every rank must make the same choice (same number of passes, same collectives)
            t = torch.tensor([k], device=self.env.device)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            k = int(t)
        logger.info(f"gradient accumulation: up to {k} micro-batches ({k * step1_tokens} padded tokens) per "
                    f"forward/backward pass (activations ~{act / 2**30:.1f} GiB per micro-batch, base "
                    f"{base_bytes / 2**30:.1f} GiB)")
        return k * step1_tokens if k > 1 else None

    @staticmethod
    def _merge(group, pad_id: int):
        """Concatenate micro-batches along the batch dim, padding sequence dims to the group max (input / decoder ids
        with the pad token, masks with 0, labels with -100 — what the collator would have produced for one batch)."""
        if len(group) == 1:
            return group[0]
        fill = {"labels": -100, "attention_mask": 0, "decoder_attention_mask": 0}
        out, padded = {}, False
        for k in group[0]:
            ts = [g[k] for g in group]
            if ts[0].dim() >= 2 and len({t.shape[1] for t in ts}) > 1:
                n = max(t.shape[1] for t in ts)
                ts = [torch.nn.functional.pad(t, (0, n - t.shape[1]), value=fill.get(k, pad_id)) for t in ts]
                padded = True
            out[k] = torch.cat(ts, 0)
        if padded and "labels" in out:  # shift_right(labels) inside the model rebuilds them for the longer labels
            out.pop("decoder_input_ids", None)
        return out

    def _to_device(self, batch, cp=False):
        nb = self.env.device.type == "cuda"
        out = {k: v.to(self.env.device, non_blocking=nb) for k, v in batch.items() if torch.is_tensor(v)}
        if cp and self.cp_group is not None:  # this rank's slice of the encoder sequence
            for k in ("input_ids", "attention_mask"):
                if k in out:
                    out[k] = shard_sequence(out[k], self.cp_group).contiguous()
        return out

    # ------------------------------------------------------------------ main loop
    def train(self, resume_from_checkpoint: str | bool | None = None):
        args, eng, env = self.args, self.engine, self.env
        _, probe = self._loader(self.train_dataset, args.per_device_train_batch_size, True)
        # an epoch's last optimizer step takes the leftover micro-batches (HF Trainer: ceil(len / ga) updates)
        steps_per_epoch = max(1, math.ceil(len(probe) / args.gradient_accumulation_steps))
        if args.max_steps > 0:
            max_steps = args.max_steps
            epochs = math.ceil(max_steps / steps_per_epoch)
        else:
            epochs = math.ceil(args.num_train_epochs)
            max_steps = math.ceil(args.num_train_epochs * steps_per_epoch)
        warmup = args.warmup_steps or int(math.ceil(args.warmup_ratio * max_steps))
        self.scheduler = LRScheduler(eng.optimizer, args.lr_scheduler_type, warmup, max_steps)
        self.state.max_steps = max_steps
        self.state.num_train_epochs = epochs
        start_epoch, skip = 0, 0
        step_seed_start = None
        resume = resume_from_checkpoint if resume_from_checkpoint is not None else args.resume_from_checkpoint
        if resume:
            path = latest_checkpoint(args.output_dir) if resume is True else resume
            if path:
                info = load_checkpoint(path, self.model, eng.optimizer, self.scheduler, rank=env.rank)
                ts = info.get("trainer_state", {})
                self.state.global_step = ts.get("global_step", 0)
                self.state.coalesce_cap = ts.get("coalesce_cap")
                self.state.coalesce_cap_unit = ts.get("coalesce_cap_unit")
                self.state.log_history = ts.get("log_history", [])
                step_seed_start = info.get("step_seed")
                start_epoch = self.state.global_step // steps_per_epoch
                skip = (self.state.global_step % steps_per_epoch) * args.gradient_accumulation_steps
                logger.info(f"resumed from {path} at step {self.state.global_step}")
        n_examples = len(self.train_dataset)
        self.handler.fire("on_train_begin", args, self.state, self.control)
        eng.train()
        t_start = time.perf_counter()
        tr_loss_sum = torch.zeros((), device=env.device)
        tr_loss_n = torch.zeros((), device=env.device)
        total_loss_sum, total_loss_n = 0.0, 0
        last_norm = None
        ga = args.gradient_accumulation_steps
        cap = self._coalesce_cap()
        cap_units = "micro" if cap is not None and cap > 0 else "tokens"
        if cap is not None and self.state.coalesce_cap is not None:  # resumed: the original run's budget, same unit
            if self.state.coalesce_cap_unit == "padded_tokens":
                cap, cap_units = (self.state.coalesce_cap or None), "tokens"
            elif self.state.coalesce_cap:  # legacy checkpoint: a budget in samples, converted at the first group
                cap, cap_units = self.state.coalesce_cap, "samples"
            else:
                cap = None
        pad_id = getattr(getattr(self.model, "config", None), "pad_token_id", 0) or 0
        # the optimizer step (passes + sync + clip + AdamW) replayed from HIP graphs once batch shapes repeat
        # (train/graph.py StepRunner; the reference pads to max_length, so every full step has one shape); context
        # parallelism keeps its eager ring-attention collectives
        runner = StepRunner(eng, enabled=graphs_enabled(env.device) and self.cp_group is None, num_items=True,
                            dp_ranks=self.dp_world)
        if runner.enabled and step_seed_start is not None:
            eng.enable_step_seeds(step_seed_start)
        self.step_runner = runner
        # first JSON line: the communication design of this run (bucket size and how it was chosen, schedules)
        self.log({"comm": runner.comm_report()})
        self._batch_shape = None
        if cap == -1:
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats(env.device)
            mem_base = torch.cuda.memory_allocated(env.device)
            # the measured step runs micro-batch by micro-batch WITHOUT deferred weight gradients (ops/gemm.py
            # WgradDefer), whose kept operands would otherwise count as one micro-batch's activations
            eng.defer_enabled = False
        warm_step = self.state.global_step + min(2, max(0, max_steps - self.state.global_step - 1))
        captured_at = None
        t_warm = t_last = None
        for epoch in range(start_epoch, epochs):
            loader, sampler = self._loader(self.train_dataset, args.per_device_train_batch_size, True, epoch)
            self.handler.fire("on_epoch_begin", args, self.state, self.control)
            n_micro = len(loader)
            it = iter(loader)
            for _ in range(skip if epoch == start_epoch else 0):
                next(it)
            done = skip if epoch == start_epoch else 0
            while done < n_micro:
                # one optimizer step = the next ga micro-batches (fewer at the end of the epoch), normalised by
                # their global non-ignored target-token count (one int64 all-reduce per step)
                group = [self._to_device(next(it), cp=True) for _ in range(min(ga, n_micro - done))]
                if self._batch_shape is None:
                    b0 = group[0]
                    self._batch_shape = [int(b0["labels"].shape[0]), int(b0["input_ids"].shape[1]),
                                         int(b0["labels"].shape[1])]
                done += len(group)
                num_items = sum(token_count(b["labels"]) for b in group)
                if self.dp_world > 1:
                    dist.all_reduce(num_items)
                    if self.cp_group is not None:  # every CP rank of a DP group counted the same batch
                        num_items = num_items // (self.env.world_size // self.dp_world)
                passes = [[b] for b in group]
                if cap is not None and cap > 0 and cap_units in ("micro", "samples"):
                    # explicit setting (k micro-batches) or a legacy sample budget -> padded tokens at this group's
                    # lengths, recorded so that a resumed run groups its passes exactly like this one
                    per = self._padded_tokens(group[:1])
                    if cap_units == "samples":
                        per = per // max(1, group[0]["labels"].shape[0])
                    cap, cap_units = cap * per, "tokens"
                    self.state.coalesce_cap, self.state.coalesce_cap_unit = cap, "padded_tokens"
                if cap is not None and cap > 0:  # coalesced: consecutive micro-batches, <= cap padded tokens per pass
                    passes, cur = [], []
                    for b in group:
                        if cur and self._padded_tokens(cur + [b]) > cap:
                            passes.append(cur)
                            cur = []
                        cur.append(b)
                    passes.append(cur)
                losses, last_norm = runner([self._merge(pb, pad_id) for pb in passes], num_items=num_items,
                                           lr=self.scheduler.get_last_lr()[0])
                for pb, loss in zip(passes, losses):
                    # logged loss: token-weighted mean (sum of token losses / tokens), the same number whether the
                    # micro-batches run one by one or merged into passes of different token counts
                    ntok = sum(token_count(b["labels"]) for b in pb).float()
                    tr_loss_sum += loss.float() * ntok
                    tr_loss_n += ntok
                if cap == -1:  # decide from the first (uncoalesced) step's measured activation memory
                    torch.cuda.synchronize()
                    cap = self._auto_cap(mem_base, torch.cuda.max_memory_allocated(env.device),
                                         max(self._padded_tokens([b]) for b in group))
                    self.state.coalesce_cap, self.state.coalesce_cap_unit = cap or 0, "padded_tokens"
                    eng.defer_enabled = True
                self.scheduler.step()
                self.state.global_step += 1
                if runner.replays and captured_at is None:  # the step that captured the HIP graph is warm-up too
                    captured_at = self.state.global_step
                    if captured_at < max_steps:
                        warm_step = max(warm_step, captured_at)
                if self.state.global_step in (warm_step, max_steps):  # steady-state clock: after the first steps,
                    if env.device.type == "cuda":                      # before the final eval / checkpoint
                        torch.cuda.synchronize()
                    if self.state.global_step == warm_step:
                        t_warm = time.perf_counter()
                    else:
                        t_last = time.perf_counter()
                self.state.epoch = epoch + done / max(1, n_micro)
                self.control = self.handler.fire("on_step_end", args, self.state, self.control)
                if self.control.should_log:
                    nt = float(tr_loss_n)
                    mean = collectives.mean_across_processes({"loss": float(tr_loss_sum) / max(1.0, nt)},
                                                             env.device)["loss"]
                    total_loss_sum += mean * nt
                    total_loss_n += nt
                    tr_loss_sum.zero_()
                    tr_loss_n.zero_()
                    if args.nan_guard and not math.isfinite(mean):  # NaN/Inf guard on loss
                        raise FloatingPointError(f"non-finite training loss {mean} at step {self.state.global_step}")
                    self.log({"loss": round(mean, 4), "grad_norm": float(last_norm) if last_norm is not None else None,
                              "learning_rate": self.scheduler.get_last_lr()[0], "epoch": round(self.state.epoch, 4)})
                if self.control.should_evaluate and self.eval_dataset is not None:
                    self.evaluate()
                    eng.train()
                if self.control.should_save:
                    self._save_checkpoint()
                faults.maybe_inject(self.state.global_step, env.rank)
                self.control.reset_step()
                if self.state.global_step >= max_steps:
                    break
            self.control = self.handler.fire("on_epoch_end", args, self.state, self.control)
            if self.state.global_step >= max_steps:
                break
        nt = float(tr_loss_n)
        if nt > 0:
            mean = collectives.mean_across_processes({"loss": float(tr_loss_sum) / nt}, env.device)["loss"]
            total_loss_sum += mean * nt
            total_loss_n += nt
        if env.device.type == "cuda":
            torch.cuda.synchronize()
        runtime = time.perf_counter() - t_start
        train_loss = total_loss_sum / max(1, total_loss_n)
        n_samples = n_examples * args.num_train_epochs if args.max_steps <= 0 else \
            max_steps * args.per_device_train_batch_size * ga * self.dp_world
        metrics = {"train_runtime": round(runtime, 4), "train_samples_per_second": round(n_samples / runtime, 3),
                   "train_steps_per_second": round(self.state.global_step / runtime, 3),
                   "train_loss": train_loss, "epoch": round(self.state.epoch, 4)}
        if t_warm is not None and t_last is not None and self.state.global_step > warm_step:
            # loop throughput without the first steps (allocator / kernel warm-up) and without the final evaluation /
            # checkpoint: the number comparable with bench.py
            per_step = args.per_device_train_batch_size * ga * self.dp_world
            dt = t_last - t_warm
            metrics["train_steady_samples_per_second"] = round(per_step * (self.state.global_step - warm_step) / dt, 3)
        if self._batch_shape is not None:  # what the throughput was measured on: per-GPU micro-batch, padded lengths
            metrics["batch_shape"] = self._batch_shape
            metrics["hip_graph_replays"] = self.step_runner.replays
            if self.step_runner.decision is not None:  # auto policy's probe: graph kept iff not slower than eager
                metrics["hip_graph_decision"] = self.step_runner.decision
        self.log(metrics)
        self.handler.fire("on_train_end", args, self.state, self.control)
        return TrainOutput(self.state.global_step, train_loss, metrics)

    def log(self, logs: dict):
        logs = {k: v for k, v in logs.items() if v is not None}
        self.state.log_history.append({**logs, "step": self.state.global_step})
        self.handler.fire("on_log", self.args, self.state, self.control, logs=logs)

    @torch.no_grad()
    def evaluate(self, eval_dataset=None):
        ds = eval_dataset if eval_dataset is not None else self.eval_dataset
        self.engine.train(False)
        # evaluation shards samples over every rank, full sequences (no context parallelism)
        loader, _ = self._loader(ds, self.args.per_device_eval_batch_size, False, cp=False)
        tot = torch.zeros((), device=self.env.device, dtype=torch.float64)
        n = 0
        if self.cp_group is not None:
            self.model.enable_context_parallel(enable=False)
        try:
            for batch in loader:
                out = self.engine.forward(self._to_device(batch))
                tot += out.loss.double()
                n += 1
        finally:
            if self.cp_group is not None:
                self.model.enable_context_parallel(self.cp_group)
        m = collectives.mean_across_processes({"eval_loss": float(tot) / max(1, n)}, self.env.device)
        metrics = {"eval_loss": m["eval_loss"], "epoch": round(self.state.epoch, 4)}
        self.log(metrics)
        self.handler.fire("on_evaluate", self.args, self.state, self.control, metrics=metrics)
        return metrics

    def _save_checkpoint(self):
        path = os.path.join(self.args.output_dir, f"checkpoint-{self.state.global_step}")
        save_checkpoint(path, self.model, self.engine.optimizer, self.scheduler, self.state, rank=self.env.rank,
                        device=self.env.device)
        if self.env.is_main_process and self.tokenizer is not None and hasattr(self.tokenizer, "save_pretrained"):
            self.tokenizer.save_pretrained(path)
        self.handler.fire("on_save", self.args, self.state, self.control)
        if self.args.save_total_limit and self.env.is_main_process:
            import shutil
            cks = sorted((d for d in os.listdir(self.args.output_dir) if d.startswith("checkpoint-")),
                         key=lambda d: int(d.split("-")[1]))
            for d in cks[: max(0, len(cks) - self.args.save_total_limit)]:
                shutil.rmtree(os.path.join(self.args.output_dir, d), ignore_errors=True)

    def save_model(self, output_dir=None):
        from ..platform.valohai import save_valohai_metadata
        return save_valohai_metadata(self.model, output_dir or self.args.output_dir, self.env.is_main_process,
                                     self.tokenizer)
