#!/usr/bin/env python
"""Trainer-style fine-tuning under torchrun (counterpart of ref/train-torchrun.py).

    torchrun --nproc-per-node=8 --master-addr 127.0.0.1 train-torchrun.py --model-ckpt t5-base ...

Same six flags and defaults as the reference; the HF Trainer configuration it builds
(ref/train-torchrun.py:115-128: warmup, per-device batch, weight_decay 0.01, logging_steps 10,
eval every ``--evaluation-steps``, save_steps 1e6, gradient_accumulation_steps 16) maps onto
train/trainer.py.  Source and target are padded to the tokenizer's ``model_max_length`` as the
reference's ``convert_examples_to_features`` does (1024 for BART, 512 for T5) unless
``--max-source-length`` / ``--max-target-length`` are given.  Logs are JSON lines (PrinterCallback).
The final model is written in HF format with Valohai metadata sidecars (rank 0 only).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault("TRANSFORMERS_NO_ADVISORY_WARNINGS", "true")

from distributed_llms_example_amd.cli import base_parser, build_data, eval_batch_size, model_config  # noqa: E402
from distributed_llms_example_amd.data.collator import DataCollatorForSeq2Seq  # noqa: E402
from distributed_llms_example_amd.models import build_model, from_pretrained  # noqa: E402
from distributed_llms_example_amd.parallel.env import init_distributed  # noqa: E402
from distributed_llms_example_amd.platform import valohai  # noqa: E402
from distributed_llms_example_amd.train.callbacks import PrinterCallback  # noqa: E402
from distributed_llms_example_amd.train.trainer import Trainer, TrainingArguments  # noqa: E402
from distributed_llms_example_amd.utils.gpu_report import gpu_report  # noqa: E402
from distributed_llms_example_amd.utils.logging import get_logger, setup_logging  # noqa: E402


def run(args):
    env = init_distributed()
    setup_logging(env.is_local_main_process)
    log = get_logger("train-torchrun")
    output_dir = valohai.outputs().path(args.output_dir)
    cfg = model_config(args)
    if env.is_local_main_process:
        gpu_report(env.device, print_fn=log.info)
    mml = 1024 if cfg.model_type == "bart" else 512
    if args.max_source_length is None:
        args.max_source_length = mml
    if args.max_target_length is None:
        args.max_target_length = mml
    tok, train_ds, eval_ds = build_data(args, cfg)
    if env.is_main_process:
        print(f"Train dataset size: {len(train_ds)}")
        print(f"Test dataset size: {len(eval_ds)}")
    torch.manual_seed(args.seed)  # random-init runs (no pretrained weights offline) start identically
    model = from_pretrained(args.model_ckpt) if os.path.isdir(args.model_ckpt or "") else build_model(cfg)
    if cfg.gradient_checkpointing:
        model.gradient_checkpointing_enable()
    targs = TrainingArguments(
        output_dir=output_dir, num_train_epochs=args.num_epochs, warmup_steps=args.warmup_steps,
        per_device_train_batch_size=args.batch_size, per_device_eval_batch_size=eval_batch_size(args, env.device),
        weight_decay=0.01, logging_steps=10, evaluation_strategy="steps", eval_steps=args.evaluation_steps,
        save_steps=args.save_steps or 1e6, gradient_accumulation_steps=args.grad_accum or 16, ddp_find_unused_parameters=False,
        learning_rate=args.learning_rate, max_steps=args.max_steps, seed=args.seed,
        bf16=None if args.precision is None else args.precision == "bf16",
        ddp_bucket_cap_mb=args.bucket_mb, overlap_comm=not args.no_overlap, grad_reduce_dtype=args.grad_reduce_dtype,
        context_parallel_size=args.context_parallel,
        coalesce_grad_accum=getattr(args, "coalesce_grad_accum", "auto"))
    trainer = Trainer(model=model, args=targs, tokenizer=tok, data_collator=DataCollatorForSeq2Seq.for_model(cfg),
                      train_dataset=train_ds, eval_dataset=eval_ds, callbacks=[PrinterCallback], env=env)
    resume = True if args.resume_from == "latest" else args.resume_from
    trainer.train(resume_from_checkpoint=resume)
    trainer.save_model(output_dir)
    env.barrier()


if __name__ == "__main__":
    p = base_parser("Train a Seq2Seq model")
    p.set_defaults(max_source_length=None, max_target_length=None)
    run(p.parse_args())
