#!/usr/bin/env python
"""Accelerate-style custom training loop (counterpart of ref/train-accelerator.py).

    torchrun --nproc-per-node=8 --master-addr 127.0.0.1 train-accelerator.py --model-ckpt facebook/bart-large-cnn

The loop is the reference's (ref/train-accelerator.py:142-280): AdamW lr 5e-5 with weight decay 0.0
in both groups, linear schedule with 1 warmup step over ``len(train_dl) * epochs`` steps, log
``{"loss", "step"}`` every 300 steps, per-epoch beam-search eval (``max_length=128, num_beams=2``),
predictions padded/gathered across ranks, ROUGE with stemming, metrics averaged across ranks, save at
the end.  ``accelerator.prepare`` maps it onto the native runtime (fused kernels, flat-buffer RCCL
reducer, fused AdamW).  Deviation: ``--batch-size`` is honoured (the reference hard-codes 1;
the default is still 1), SURVEY.md Appendix A Q4.
"""
import json
import time
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault("TRANSFORMERS_NO_ADVISORY_WARNINGS", "true")

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402

from distributed_llms_example_amd.cli import base_parser, build_data, eval_batch_size, model_config  # noqa: E402
from distributed_llms_example_amd.data.collator import DataCollatorForSeq2Seq  # noqa: E402
from distributed_llms_example_amd.models import build_model, from_pretrained  # noqa: E402
from distributed_llms_example_amd.utils import faults  # noqa: E402
from distributed_llms_example_amd.ops.rng import manual_seed  # noqa: E402
from distributed_llms_example_amd.platform import valohai  # noqa: E402
from distributed_llms_example_amd.train import rouge  # noqa: E402
from distributed_llms_example_amd.train.accelerator import Accelerator, get_scheduler  # noqa: E402
from distributed_llms_example_amd.utils.gpu_report import gpu_report  # noqa: E402
from distributed_llms_example_amd.utils.logging import get_logger, setup_logging  # noqa: E402


class ModelTrainer:
    def __init__(self, args):
        self.args = args
        mp = None if args.precision is None else ("bf16" if args.precision == "bf16" else "no")
        self.accelerator = Accelerator(mixed_precision=mp, bucket_mb=args.bucket_mb or "auto",
                                       overlap_comm=not args.no_overlap, seed=args.seed,
                                       grad_reduce_dtype=args.grad_reduce_dtype)
        self.device = self.accelerator.device
        setup_logging(self.accelerator.is_local_main_process)
        self.logger = get_logger("train-accelerator")
        self.logger.info(self.accelerator.state)
        if self.accelerator.is_local_main_process:
            gpu_report(self.device, print_fn=self.logger.info)
        torch.manual_seed(args.seed)
        manual_seed(args.seed + 7919 * self.accelerator.process_index)
        self.cfg = model_config(args)
        self.model = from_pretrained(args.model_ckpt) if os.path.isdir(args.model_ckpt or "") else \
            build_model(self.cfg)
        if self.cfg.gradient_checkpointing:
            self.model.gradient_checkpointing_enable()

    def dump(self, logs):
        if self.accelerator.is_main_process:
            print(json.dumps(logs), flush=True)

    def train(self, output_dir, tokenizer, train_ds, eval_ds):
        a, acc = self.args, self.accelerator
        collator = DataCollatorForSeq2Seq.for_model(self.cfg)
        train_dl = DataLoader(train_ds, shuffle=True, collate_fn=collator, batch_size=a.batch_size)
        eval_dl = DataLoader(eval_ds, collate_fn=collator, batch_size=eval_batch_size(a, self.accelerator.device))
        no_decay = ["bias", "LayerNorm.weight"]
        groups = [
            {"params": [p for n, p in self.model.named_parameters() if not any(nd in n for nd in no_decay)],
             "weight_decay": 0.0},
            {"params": [p for n, p in self.model.named_parameters() if any(nd in n for nd in no_decay)],
             "weight_decay": 0.0},
        ]
        optimizer = torch.optim.AdamW(groups, lr=a.learning_rate)
        model, optimizer, train_dl, eval_dl = acc.prepare(self.model, optimizer, train_dl, eval_dl)
        max_train_steps = a.num_epochs * len(train_dl)
        if a.max_steps > 0:
            max_train_steps = min(max_train_steps, a.max_steps)
        lr_scheduler = get_scheduler("linear", optimizer, num_warmup_steps=1, num_training_steps=max_train_steps)
        metric = rouge.load("rouge")
        train_step = acc.make_train_step(model, optimizer)
        self.dump({"comm": train_step.runner.comm_report()})  # bucket choice and step schedules of this run
        self.logger.info(f"***** Running training ***** examples={len(train_ds)} epochs={a.num_epochs}")
        completed = 0
        shape = None
        t0 = time.perf_counter()
        t_warm, warm = None, min(2, max(0, max_train_steps - 1))
        for epoch in range(a.num_epochs):
            model.train()
            train_dl.set_epoch(epoch)
            for batch in train_dl:
                # == outputs = model(**batch); acc.backward(outputs.loss); optimizer.step(); optimizer.zero_grad()
                # (ref/train-accelerator.py:219-228), replayed from a HIP graph on GPU once the batch shape repeats
                loss = train_step(batch)
                lr_scheduler.step()
                completed += 1
                shape = [int(batch["input_ids"].shape[1]), int(batch["labels"].shape[1])]
                if train_step.runner.replays == 1 and completed < max_train_steps:
                    warm = completed  # the step that captured the HIP graph is warm-up too
                if completed == warm:
                    torch.cuda.synchronize() if acc.device.type == "cuda" else None
                    t_warm = time.perf_counter()
                faults.maybe_inject(completed, acc.process_index)
                if completed % 300 == 0:
                    self.dump({"loss": loss.item(), "step": completed})
                if completed >= max_train_steps:
                    break
            torch.cuda.synchronize() if acc.device.type == "cuda" else None
            t1 = time.perf_counter()
            per_step = a.batch_size * acc.num_processes
            tp = {"train_samples_per_second": round(per_step * completed / (t1 - t0), 3), "epoch": epoch,
                  "batch_shape": [a.batch_size] + (shape or []),  # per-GPU batch, padded source / target tokens
                  "hip_graph_replays": train_step.runner.replays}
            if train_step.runner.decision is not None:
                tp["hip_graph_decision"] = train_step.runner.decision
            if t_warm is not None and completed > warm:
                tp["train_steady_samples_per_second"] = round(per_step * (completed - warm) / (t1 - t_warm), 3)
            self.dump(tp)
            model.eval()
            for batch in eval_dl:
                with torch.no_grad():
                    gen = acc.unwrap_model(model).generate(batch["input_ids"], attention_mask=batch["attention_mask"],
                                                           max_length=a.gen_max_length, num_beams=a.num_beams)
                    gen = acc.pad_across_processes(gen, dim=1, pad_index=tokenizer.pad_token_id)
                    labels = acc.pad_across_processes(batch["labels"], dim=1, pad_index=-100)
                    gen = acc.gather(gen).cpu().numpy()
                    labels = acc.gather(labels).cpu().numpy()
                    labels = np.where(labels != -100, labels, tokenizer.pad_token_id)
                    preds = tokenizer.batch_decode(gen, skip_special_tokens=True)
                    refs = tokenizer.batch_decode(labels, skip_special_tokens=True)
                    metric.add_batch(predictions=preds, references=refs)
            metrics = metric.compute(use_stemmer=True)
            self.dump(acc.reduce_mean(metrics))
        if output_dir is not None:
            acc.wait_for_everyone()
            acc.save_model(model, output_dir)
            acc.wait_for_everyone()


def run(args):
    output_dir = valohai.outputs().path(args.output_dir)
    mt = ModelTrainer(args)
    tok, train_ds, eval_ds = build_data(args, mt.cfg)
    if mt.accelerator.is_main_process:
        print(f"Train dataset size: {len(train_ds)}")
        print(f"Test dataset size: {len(eval_ds)}")
    mt.train(output_dir, tok, train_ds, eval_ds)


if __name__ == "__main__":
    args = base_parser("Train a Seq2Seq model").parse_args()
    if args.context_parallel > 1:
        raise SystemExit("--context-parallel is implemented in train-torchrun.py (Trainer path)")
    run(args)
