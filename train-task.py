#!/usr/bin/env python
"""Multi-machine data-parallel training via torch.multiprocessing + TCP rendezvous
(counterpart of ref/train-task.py).

Reference flow (ref/train-task.py:404-430): every Valohai execution (one per machine) reads the
master IP / world size / rank from the Valohai distributed API, spawns ONE child with
``mp.set_start_method('spawn')``, which calls ``init_process_group('tcp://<master>:1234', backend=nccl)``
and trains on its ``DataPartitioner`` shard (seed 1234) with per-tensor ``all_reduce`` + divide.

Here the same launch contract is kept, plus ``--local-procs N`` to run N ranks on one node (one per
GPU — BASELINE.json's "t5-large train-task torch.multiprocessing spawn, 8 RCCL ranks on one node").
Gradient averaging is the coalesced flat-buffer all-reduce (same math as the per-tensor loop, one RCCL
call instead of ~500), overlapped with backward by default (``--no-overlap``: after backward).  Deviations
(SURVEY.md Appendix A Q4/Q9): ``--batch-size`` is honoured (the reference uses ceil(2/world)); the
eval set is sharded and gathered instead of decoded redundantly on every rank — the aggregated
ROUGE is the same; loss is synced to the host only at log steps.
"""
import argparse
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault("TRANSFORMERS_NO_ADVISORY_WARNINGS", "true")

import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from distributed_llms_example_amd.cli import base_parser, eval_batch_size  # noqa: E402
from distributed_llms_example_amd.platform import valohai  # noqa: E402


def init(rank, world, url, args, local_index=0):
    """Child process: rendezvous, then run."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    os.environ["LOCAL_RANK"] = str(local_index)
    from distributed_llms_example_amd.parallel.env import init_distributed
    cpu = not torch.cuda.is_available() or os.environ.get("DLLM_FORCE_CPU") == "1"
    env = init_distributed(init_method=url, rank=rank, world_size=world, cpu=cpu)
    try:
        run(env, args)
    finally:
        from distributed_llms_example_amd.parallel.env import shutdown
        shutdown()


def run(env, args):
    import numpy as np
    from torch.utils.data import DataLoader

    from distributed_llms_example_amd.cli import build_data, model_config
    from distributed_llms_example_amd.data.collator import DataCollatorForSeq2Seq
    from distributed_llms_example_amd.models import build_model, from_pretrained
    from distributed_llms_example_amd.ops.rng import manual_seed
    from distributed_llms_example_amd.parallel import collectives
    from distributed_llms_example_amd.parallel.sampler import DataPartitioner, ShardedBatchSampler
    from distributed_llms_example_amd.train import rouge
    from distributed_llms_example_amd.utils import faults
    from distributed_llms_example_amd.train.engine import TrainEngine
    from distributed_llms_example_amd.train.graph import StepRunner
    from distributed_llms_example_amd.train.schedule import LRScheduler
    from distributed_llms_example_amd.utils.gpu_report import gpu_report
    from distributed_llms_example_amd.utils.logging import dump_metrics, get_logger, setup_logging

    setup_logging(env.is_local_main_process)
    log = get_logger("train-task")
    output_dir = valohai.outputs().path(args.output_dir)
    cfg = model_config(args)
    if env.is_local_main_process:
        gpu_report(env.device, print_fn=log.info)
    torch.manual_seed(args.seed)
    manual_seed(args.seed + 7919 * env.rank)
    tok, train_ds, eval_ds = build_data(args, cfg)
    if env.is_main_process:
        print(f"Train dataset size: {len(train_ds)}")
        print(f"Test dataset size: {len(eval_ds)}")
    model = from_pretrained(args.model_ckpt) if os.path.isdir(args.model_ckpt or "") else build_model(cfg)
    if cfg.gradient_checkpointing:
        model.gradient_checkpointing_enable()
    dtype = torch.bfloat16 if (args.precision or ("bf16" if env.device.type == "cuda" else "fp32")) == "bf16" \
        else torch.float32
    eng = TrainEngine(model, env, lr=args.learning_rate, weight_decay=0.0, max_grad_norm=None, dtype=dtype,
                      bucket_mb=args.bucket_mb or "auto", overlap=not args.no_overlap, no_decay=None,
                      grad_reduce_dtype=args.grad_reduce_dtype)
    collator = DataCollatorForSeq2Seq.for_model(cfg, pad_to_multiple_of=8)
    # partition_dataset (ref/train-task.py:176-191)
    world = env.world_size
    part = DataPartitioner(train_ds, [1.0 / world for _ in range(world)], seed=1234).use(env.rank)
    bsz = args.batch_size if args.batch_size else math.ceil(2 / float(world))
    train_dl = DataLoader(part, batch_size=bsz, shuffle=True, collate_fn=collator)
    ev_sampler = ShardedBatchSampler(len(eval_ds), eval_batch_size(argparse.Namespace(**{**vars(args), "batch_size": bsz}), env.device),
                                     world, env.rank)
    eval_dl = DataLoader(eval_ds, batch_sampler=ev_sampler, collate_fn=collator)
    max_steps = args.num_epochs * len(train_dl)
    if args.max_steps > 0:
        max_steps = min(max_steps, args.max_steps)
    sched = LRScheduler(eng.optimizer, "linear", 1, max_steps)
    metric = rouge.load("rouge")
    dev = env.device
    # forward + backward + gradient all-reduce + AdamW, replayed from HIP graphs once the batch shape repeats
    # (train/graph.py StepRunner; eager on CPU, DLLM_GRAPH=0, or for a ragged last batch)
    runner = StepRunner(eng)
    dump_metrics({"comm": runner.comm_report()}, env.is_main_process)  # bucket choice and step schedules of this run
    completed = 0
    for epoch in range(args.num_epochs):
        eng.train()
        loss_acc = torch.zeros((), device=dev)
        for batch in train_dl:
            batch = {k: v.to(dev, non_blocking=True) for k, v in batch.items()}
            # all-reduce of the flat gradient buffer (average_gradients, ref/train-task.py:65-69,293) + AdamW
            losses, _ = runner([batch], lr=sched.get_last_lr()[0])
            loss = losses[0]
            loss_acc += loss
            sched.step()
            completed += 1
            faults.maybe_inject(completed, env.rank)
            if completed % 100 == 0:
                dump_metrics({"loss": float(loss), "step": completed}, env.is_main_process)
            if completed >= max_steps:
                break
        eng.train(False)
        for batch in eval_dl:
            batch = {k: v.to(dev) for k, v in batch.items()}
            with torch.no_grad():
                gen = eng.model.generate(batch["input_ids"], attention_mask=batch["attention_mask"],
                                         max_length=args.gen_max_length, num_beams=args.num_beams)
            gen = collectives.pad_across_processes(gen, dim=1, pad_index=tok.pad_token_id)
            labels = collectives.pad_across_processes(batch["labels"], dim=1, pad_index=-100)
            gen = collectives.gather(gen).cpu().numpy()
            labels = collectives.gather(labels).cpu().numpy()
            labels = np.where(labels != -100, labels, tok.pad_token_id)
            metric.add_batch(predictions=tok.batch_decode(gen, skip_special_tokens=True),
                             references=tok.batch_decode(labels, skip_special_tokens=True))
        result = {k: round(v * 100, 4) for k, v in metric.compute(use_stemmer=True).items()}
        result["epoch"] = epoch
        avg = collectives.mean_across_processes(result, dev)
        if env.is_main_process:
            print("Metrics aggregated across all machines: ")
        dump_metrics(avg, env.is_main_process)
        if completed >= max_steps:  # --max-steps: no further epochs (each would run a step and a full eval)
            break
    if output_dir is not None:
        env.barrier()
        from distributed_llms_example_amd.platform.valohai import save_valohai_metadata
        save_valohai_metadata(eng.model, output_dir, env.is_main_process)
        env.barrier()


def main():
    p = base_parser("Train a Seq2Seq model", defaults={"batch_size": 6})
    p.add_argument("--local-procs", type=int, default=0, help="spawn N ranks on this node (one per GPU)")
    p.add_argument("--master-port", type=int, default=1234)
    p.add_argument("--overlap", action="store_true",
                   help="(default) overlap the bucketed gradient all-reduce with backward; --no-overlap: one coalesced "
                        "all-reduce after backward, the ref/train-task.py:65-69 call pattern (same math)")
    args = p.parse_args()
    if getattr(args, "context_parallel", 1) > 1:
        raise SystemExit("--context-parallel is implemented in train-torchrun.py (Trainer path)")
    mp.set_start_method("spawn", force=True)
    if args.local_procs and args.local_procs > 0:
        url = f"tcp://127.0.0.1:{args.master_port}"
        procs = []
        for r in range(args.local_procs):
            pr = mp.Process(target=init, args=(r, args.local_procs, url, args, r))
            pr.start()
            procs.append(pr)
        rc = 0
        for pr in procs:
            pr.join()
            rc = rc or pr.exitcode
        sys.exit(rc)
    master_ip = valohai.distributed.master().primary_local_ip
    url = f"tcp://{master_ip}:{args.master_port}"
    world = valohai.distributed.required_count
    rank = valohai.distributed.me().rank
    p0 = mp.Process(target=init, args=(rank, world, url, args, 0))
    p0.start()
    p0.join()
    sys.exit(p0.exitcode)


if __name__ == "__main__":
    main()
