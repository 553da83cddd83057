#!/usr/bin/env python
"""Headline benchmark: whole-node samples/sec of T5-base summarization fine-tuning (BASELINE.json).

One process per GPU (torchrun sets RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*; N=1 runs standalone), data
parallel over RCCL with the bucketed reducer, bf16 weights/activations with fp32 master weights and
moments, full training step inside the timed region: encoder+decoder forward, fused CE loss,
backward, gradient all-reduce, global-norm clip and AdamW update.  Synthetic SAMSum-shaped data
(input 1024 / target 128 tokens, the ref/train-accelerator.py:114-133 shapes) and random-init
weights with HF's initialisation (no network).  Weak scaling: fixed per-GPU micro-batch.

    python bench.py --gpus N --steps K --warmup W

``--gpus N > 1`` without a launcher (no WORLD_SIZE in the environment) starts its own: the same command line under
``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1`` as a CHILD process (no exec,
and before anything touches the GPU), forwards its exit code, and rank 0 of the child prints the JSON line.  The
driver's ``torch.distributed.run ... bench.py --gpus N`` form runs the ranks directly.

Every N runs the same step: forward + backward (+ GA micro-steps) and the optimizer replayed from HIP graphs
(train/graph.py).  For N > 1 the backward graph is a chain of segments cut at the reducer's bucket boundaries and
each bucket's async RCCL all-reduce is launched between the segment replays, overlapping the rest of the backward
(``comm.schedule`` = "overlap-graph"; ``--no-overlap``: every bucket after the backward, "split-graph").  ``--graph
off`` gives the eager, hook-overlapped reducer.  ``--bucket-mb auto`` (default for N > 1) picks the bucket size from an
all-reduce probe on the job's process group (``comm.bucket_choice``); ``--grad-reduce-dtype bf16`` puts bf16 on the
wire (fp32 accumulation kept).

Multi-GPU self-diagnosis (N > 1; every field is also produced on a gloo CPU rehearsal, DLLM_FORCE_CPU=1):
  * before timing, every rank's world size, RCCL version, bucket layout (bounds + segment sizes) and parameter count
    are all-gathered and compared: a mismatch aborts the run with the differing ranks named;
  * ``comm.exposed_ms_per_step``: per synchronised backward, the time between the last backward kernel and the last
    bucket all-reduce completing on the compute stream (GPU events around the reducer's end-of-backward wait) — the
    communication NOT hidden under backward; ``comm.exposed_frac`` = that / ms_per_step;
  * ``comm.bucket_launch``: the last backward's bucket launch order and, per launch, the fraction of gradient
    segments already ready (overlap works when early buckets launch at small fractions);
  * ``--comm-stress``: per-GPU micro-batch 8 (unless --batch-per-gpu is given), so all-reduce time is comparable to
    compute and the 1->N curve measures the reducer's overlap, not just weak-scaled compute;
  * ``--grad-accum G``: G micro-batches per optimizer step, ``no_sync`` on all but the last (reference
    train-torchrun: batch 1 x GA 16, ref/train-torchrun.py:119,126); never coalesced into one pass here.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Reference stack (HF transformers T5 + torch fused AdamW, bf16 autocast, SDPA) measured on one MI355X
# with tools/hf_comparator.py at the same shapes: profiles/hf_comparator_t5base_mi355x.jsonl.
# BASELINE.md publishes no number, so vs_baseline compares against this comparator scaled linearly
# with N (an upper bound for the reference's own scaling).
HF_COMPARATOR_SAMPLES_PER_S_1GPU = {16: 107.4, 32: 132.0, 64: 150.7, 128: 155.3}
# the same stack in fp32 (the reference's own precision: no AMP configured, ref/train-torchrun.py:115-128)
HF_COMPARATOR_FP32_SAMPLES_PER_S_1GPU = {16: 76.7}
# other BASELINE.json configs, same comparator tool (profiles/configs/hf_*.json): (model, per-GPU batch) -> samples/s
HF_COMPARATOR_OTHER = {("bart-large", 32): 269.7, ("t5-large", 16): 46.6, ("flan-t5-xl", 8): 16.2}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="t5-base")
    ap.add_argument("--batch-per-gpu", type=int,
                    default=int(os.environ["DLLM_BENCH_BATCH"]) if "DLLM_BENCH_BATCH" in os.environ else None,
                    help="per-GPU micro-batch, sized for the 288 GB HBM.  Default: t5-base 512 (182 GB, +1.0 %% "
                         "samples/s over 256 in an interleaved sweep, profiles/r3_bench_batch_sweep.txt; 256: +1.9 %% over "
                         "128, profiles/r2_bench_batch_ab.txt), other models 256.  The HF comparator was measured at "
                         "16/32/64/128 — it needs 262 GB at 128, so 128 is its largest batch")
    ap.add_argument("--src-len", type=int, default=1024)
    ap.add_argument("--tgt-len", type=int, default=128)
    ap.add_argument("--bucket-mb", default="auto",
                    help="all-reduce bucket MiB, or auto (probe over 32-256 MiB on the job's process group; N > 1)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="all-reduce every bucket after the backward (graph: split schedule; eager: one coalesced call)")
    ap.add_argument("--grad-reduce-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="dtype of the gradient all-reduce on the wire (fp32 accumulation either way)")
    ap.add_argument("--dropout", type=float, default=None, help="override model dropout (default: config 0.1)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--grad-ckpt", action="store_true", help="activation checkpointing per block")
    ap.add_argument("--grad-accum", type=int, default=1, help="micro-batches per optimizer step (no_sync on all but the "
                                                               "last; samples/s counts every micro-batch)")
    ap.add_argument("--comm-stress", action="store_true",
                    help="small per-GPU batch (8 unless --batch-per-gpu is given): all-reduce ~ compute")
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="replay the step (forward, backward, GA micro-steps, clip, AdamW) from HIP graphs "
                         "(train/graph.py; N > 1: the bucketed all-reduce between the two graphs); auto: on whenever "
                         "the ranks run on GPUs; off: eager steps with the hook-overlapped reducer")
    ap.add_argument("--graph-comm", default=None, choices=["overlap", "split", "capture"],
                    help="N > 1 graph schedule (train/graph.py): overlap (default: segmented backward graph, buckets "
                         "launched between the segments), split (after backward) or capture (RCCL inside the graph)")
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp32"],
                    help="weights/activations dtype (default bf16; fp32 on a CPU rehearsal)")
    a = ap.parse_args()
    a.bucket_mb = "auto" if str(a.bucket_mb).lower() == "auto" else float(a.bucket_mb)
    if a.comm_stress and "--batch-per-gpu" not in " ".join(sys.argv):
        a.batch_per_gpu = 8
    if a.batch_per_gpu is None:
        a.batch_per_gpu = 512 if a.model == "t5-base" else 256
    return a


def _free_port() -> int:
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def self_launch(gpus: int) -> int | None:
    """``--gpus N > 1`` with no launcher around: run this same command line under torchrun as a child process (one
    rank per GPU, rendezvous on 127.0.0.1) and return its exit code.  None when already launched (WORLD_SIZE set) or
    N == 1.  Nothing here touches the GPU (counting devices does not initialise it)."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    if os.environ.get("DLLM_FORCE_CPU", "0") != "1" and os.environ.get("DLLM_DIST_BACKEND") != "gloo":
        ndev = torch.cuda.device_count()
        if ndev < gpus:
            print(f"[bench] --gpus {gpus} but only {ndev} GPU(s) visible", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] self-launch: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=dict(os.environ, DLLM_BENCH_SELF_LAUNCHED="1")).returncode


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001 - informational only
        return None


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _torch_profile(step, path: str, top: int = 60) -> None:
    """One extra (untimed) eager step under torch.profiler: device time per (kernel, Python call site), so the small
    ATen kernels in a rocprofv3 summary can be traced to the op that launched them.  Env DLLM_TORCH_PROFILE=<file>."""
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as prof:
        step(0)
        torch.cuda.synchronize()
    # library GEMMs by operand shapes (which projections still run on hipBLASLt, and at what rate)
    gemms = []
    for e in prof.key_averages(group_by_input_shape=True):
        if e.key in ("aten::mm", "aten::addmm", "aten::addmm_", "aten::bmm") and e.self_device_time_total > 0:
            gemms.append((e.self_device_time_total, e.count, e.key, str(e.input_shapes)[:120]))
    gemms.sort(reverse=True)
    rows = prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=top,
                                                       max_name_column_width=70)
    # ATen ops with their Python call sites (the rows above group by stack but do not print it)
    sites = []
    for e in prof.key_averages(group_by_stack_n=6):
        if e.key.startswith("aten::") and e.self_device_time_total > 0 and e.stack:
            sites.append((e.self_device_time_total, e.count, e.key, " <- ".join(e.stack[:6])))
    sites.sort(reverse=True)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as f:
        f.write(rows)
        f.write("\n# ATen ops by call site: self device us, calls, op, stack\n")
        for us, n, k, st in sites[:top]:
            f.write(f"{us:10.1f} {n:6d} {k:28s} {st}\n")
        f.write("\n# library GEMMs by input shapes: self device us, calls, op, shapes\n")
        for us, n, k, sh in gemms[:top]:
            f.write(f"{us:10.1f} {n:6d} {k:16s} {sh}\n")


def check_rank_consistency(env, eng, model_name: str, batch: int):
    """All-gather what every rank must agree on (RCCL matches collectives by order and size: a mismatch deadlocks or
    silently mixes gradients) and fail loudly, naming the ranks, when anything differs."""
    import hashlib
    red = eng.reducer
    sig = red.layout_signature() if red is not None else []
    mine = {"world_size": env.world_size, "rccl_version": _rccl_version() if env.backend == "nccl" else None,
            "backend": env.backend, "model": model_name, "per_gpu_batch": batch,
            "n_params": sum(p.numel() for p in eng.flat.params),
            "bucket_layout_sha": hashlib.sha1(json.dumps(sig).encode()).hexdigest()[:16],
            "n_buckets": len(red.buckets) if red is not None else 0}
    allv = [None] * env.world_size
    dist.all_gather_object(allv, mine)
    bad = {k: {r: v[k] for r, v in enumerate(allv)} for k in mine if len({json.dumps(v[k]) for v in allv}) > 1}
    if bad:
        raise SystemExit(f"[bench] rank {env.rank}: ranks disagree on {sorted(bad)}: {json.dumps(bad)}")
    return {"status": "ok", "checked": sorted(mine), **{k: mine[k] for k in ("bucket_layout_sha", "n_buckets")}}


def comm_probe(env, eng, sizes_mb=(1.0, 32.0, 128.0), iters: int = 5) -> dict:
    """In-run all-reduce bus bandwidth over the reducer's bucket sizes, fp32 and bf16 (GB/s, ring convention
    2(N-1)/N x bytes / time, the slowest rank's time): what RCCL over xGMI delivers to THIS job's buckets."""
    red = eng.reducer
    n = env.world_size
    dev = env.device if env.backend == "nccl" else torch.device("cpu")
    if dev.type == "cpu":  # gloo rehearsal: the fields, not the numbers
        sizes_mb = sizes_mb[:1]
    sizes = sorted({round(x, 2) for x in list(sizes_mb) + red.bucket_sizes_mb()[:2]})
    out = {}
    for dt in (torch.float32, torch.bfloat16):
        res = {}
        for mb in sizes:
            x = torch.ones(max(1, int(mb * 2**20) // (4 if dt == torch.float32 else 2)), dtype=dt, device=dev)
            for _ in range(2):
                dist.all_reduce(x)
            _sync(dev)
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                dist.all_reduce(x)
            _sync(dev)
            t = torch.tensor([(time.perf_counter() - t0) / iters], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            nbytes = x.numel() * x.element_size()
            res[f"{mb:g}MiB"] = round(2 * (n - 1) / n * nbytes / t.item() / 1e9, 2)
        out["fp32" if dt == torch.float32 else "bf16"] = res
    return out


def build(a, env):
    from distributed_llms_example_amd.models import build_model, resolve_config
    from distributed_llms_example_amd.ops.rng import manual_seed
    from distributed_llms_example_amd.parallel.reducer import DEFAULT_BUCKET_MB
    from distributed_llms_example_amd.train.engine import TrainEngine
    torch.manual_seed(a.seed)
    manual_seed(a.seed * 1000 + env.rank)
    cfg = resolve_config(a.model)
    if a.dropout is not None:
        cfg = cfg.replace(dropout_rate=a.dropout, attention_dropout=a.dropout)
    if a.grad_ckpt:
        cfg = cfg.replace(gradient_checkpointing=True)
    model = build_model(cfg)
    dtype_name = a.dtype or ("bf16" if env.device.type == "cuda" else "fp32")
    dtype = torch.bfloat16 if dtype_name == "bf16" else torch.float32
    bucket_mb = a.bucket_mb
    if bucket_mb == "auto" and (env.world_size == 1 or env.backend != "nccl"):
        bucket_mb = DEFAULT_BUCKET_MB  # nothing to probe (1 rank) / a gloo rehearsal: the fixed default
    eng = TrainEngine(model, env, lr=5e-5, weight_decay=0.01, max_grad_norm=1.0, dtype=dtype,
                      bucket_mb=bucket_mb, overlap=not a.no_overlap, grad_reduce_dtype=a.grad_reduce_dtype)
    eng.train()
    return cfg, eng, dtype_name


def main():
    a = parse()
    rc = self_launch(a.gpus)
    if rc is not None:
        sys.exit(rc)
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.utils.profiling import MI355X_BF16_DENSE_PEAK, seq2seq_train_flops

    env = init_distributed()
    n = env.world_size
    if a.gpus != n:
        raise SystemExit(f"[bench] --gpus {a.gpus} but WORLD_SIZE={n}: launch one rank per GPU "
                         f"(python -m torch.distributed.run --nproc-per-node {a.gpus} bench.py --gpus {a.gpus})")
    cfg, eng, dtype_name = build(a, env)
    B, S, T, V = a.batch_per_gpu, a.src_len, a.tgt_len, cfg.vocab_size
    GA = max(1, a.grad_accum)
    g = torch.Generator(device="cpu").manual_seed(1000 + env.rank)
    batches = []
    for _ in range(2 * GA):
        batches.append({
            "input_ids": torch.randint(2, V, (B, S), generator=g).to(env.device),
            "attention_mask": torch.ones(B, S, dtype=torch.long).to(env.device),
            "labels": torch.randint(2, V, (B, T), generator=g).to(env.device),
        })

    use_graph = a.graph == "on" or (a.graph == "auto" and env.device.type == "cuda")
    graphed = None
    graph_error = None
    if use_graph:
        from distributed_llms_example_amd.train.graph import GraphedStep
        try:
            graphed = GraphedStep(eng, batches[:GA], warmup=2, comm=a.graph_comm)
        except Exception as e:  # noqa: BLE001 - recorded in the JSON line; the step is then rebuilt from scratch
            if a.graph == "on" and n == 1:
                raise
            graph_error = f"{type(e).__name__}: {str(e)[:300]}"
            graphed = None
        if n > 1:
            # every rank must take the same path (graphed collective schedule vs eager hooks): agree on the capture
            # outcome before anything else runs a collective; one failed rank sends every rank to the rebuilt eager step
            ok = torch.tensor([0 if graphed is None else 1], dtype=torch.int32,
                              device=env.device if env.backend == "nccl" else "cpu")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if ok.item() == 0 and graphed is not None:
                graph_error = "capture failed on another rank"
                graphed = None
            if graphed is None and a.graph == "on":
                raise SystemExit(f"[bench] rank {env.rank}: HIP-graph capture failed ({graph_error}) with --graph on")
        if graphed is None:
            print(f"[bench] graph capture failed ({graph_error}); rebuilding the engine, eager steps", file=sys.stderr)
            torch.cuda.synchronize()
            # the failed capture left the engine mid-state (warmup steps taken, step seeds on, host mirrors ahead of
            # the device): start over with a fresh model, optimizer and seed stream
            eng.disable_step_seeds()
            if eng.reducer is not None:
                eng.reducer.remove()
            del eng
            torch.cuda.empty_cache()
            cfg, eng, dtype_name = build(a, env)

    def step(i):
        mbs = [batches[(i * GA + k) % len(batches)] for k in range(GA)]
        if graphed is not None:
            graphed.replay(mbs)
            return
        for k in range(GA):  # GA micro-batches, gradient sync (and the all-reduce) on the last only
            eng.forward_backward(mbs[k], grad_accum=GA, sync=k == GA - 1)
        eng.step()

    for i in range(a.warmup):
        step(i)
    consistency = check_rank_consistency(env, eng, a.model, B) if n > 1 else None  # after warmup: buckets rebuilt
    if eng.reducer is not None:
        eng.reducer.take_exposed_ms()
        eng.reducer.set_timing(True)
    env.barrier()
    _sync(env.device)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(i)
    env.barrier()
    _sync(env.device)
    dt = time.perf_counter() - t0
    if os.environ.get("DLLM_TORCH_PROFILE") and env.rank == 0 and graphed is None:
        _torch_profile(step, os.environ["DLLM_TORCH_PROFILE"])  # after timing: attributes kernels to call sites
    comm = None
    if eng.reducer is not None:
        eng.reducer.set_timing(False)
        ex = eng.reducer.take_exposed_ms()
        ex_t = torch.tensor([sum(ex) / max(1, len(ex)), max(ex, default=0.0)], dtype=torch.float64,
                            device=env.device if env.backend == "nccl" else "cpu")
        dist.all_reduce(ex_t, op=dist.ReduceOp.MAX)  # the slowest rank's exposure sets the step
        gcomm = graphed.comm if graphed is not None else None
        bl = eng.reducer.launch_summary()
        nb = len(eng.reducer.buckets)
        if gcomm == "split":  # every bucket launches after backward, in bucket order (GradReducer.sync_buckets)
            bl = {"order": list(range(nb)), "ready_frac_at_launch": [1.0] * nb, "launched_before_backward_end": 0,
                  "n_buckets": nb}
        elif gcomm == "overlap":  # the segmented replay: buckets launched between backward segments, then the tail
            sch = graphed.schedule()
            bl = {"order": list(range(nb)), "segments": sch["segments"], "tail_buckets": sch["tail_buckets"],
                  "launched_before_backward_end": sch["buckets_launched_before_backward_end"], "n_buckets": nb}
        comm = {"schedule": {"split": "split-graph", "overlap": "overlap-graph", "capture": "captured-graph",
                             None: "eager-overlap" if eng.reducer.overlap else "eager-post-backward"}[gcomm],
                "overlap_frac": round(bl["launched_before_backward_end"] / max(1, nb), 3),
                "grad_reduce_dtype": a.grad_reduce_dtype,
                "bucket_choice": eng.reducer.bucket_choice,
                "exposed_ms_per_step": round(ex_t[0].item(), 3), "exposed_ms_max": round(ex_t[1].item(), 3),
                "timed_backwards": len(ex), "bucket_launch": bl,
                "buckets_launched_before_backward_end": bl["launched_before_backward_end"],
                "bucket_mb": [round(x, 2) for x in eng.reducer.bucket_sizes_mb()[:4]],
                "world_size_seen_by_pg": dist.get_world_size(), "backend": dist.get_backend(),
                "rccl_version": _rccl_version() if env.backend == "nccl" else None,
                "consistency": consistency}
    t = torch.tensor([dt], device=env.device if env.backend == "nccl" else "cpu", dtype=torch.float64)
    if n > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    ms = dt / a.steps * 1e3
    value = B * GA * n * a.steps / dt
    if comm is not None:
        comm["exposed_frac"] = round(comm["exposed_ms_per_step"] / ms, 4)
        comm["busbw_gbps"] = comm_probe(env, eng)  # after the timed region: not part of the measurement
    # model FLOPs utilisation against the dense bf16 peak (2.5 PF per GPU; no 2:1-sparsity figure): analytic training
    # FLOPs of the step (GEMMs + attention + LM head, fwd + bwd = 3 x fwd; utils/profiling.py)
    step_flops = seq2seq_train_flops(cfg, B * GA, S, T)
    mfu = step_flops / (ms * 1e-3) / (MI355X_BF16_DENSE_PEAK * n)
    if a.model == "t5-base":
        metric = "samples/sec (whole node) T5-base summarization fine-tune at 1/2/4/8 MI355X"
        # the HF stack at the same per-GPU batch, or at its largest measured one below it (it does not fit above 128)
        table = HF_COMPARATOR_FP32_SAMPLES_PER_S_1GPU if dtype_name == "fp32" else HF_COMPARATOR_SAMPLES_PER_S_1GPU
        base_batch = max((bb for bb in table if bb <= B), default=None)
        base = table.get(base_batch)
    elif (a.src_len, a.tgt_len) != (1024, 128):  # comparators were measured at the 1024/128 shapes only
        metric = f"samples/sec (whole node) {a.model} summarization fine-tune, {a.src_len}/{a.tgt_len} tokens"
        base, base_batch = None, None
    else:  # per-sample throughput vs the HF stack at the batch it was measured with (noted in the line)
        metric = f"samples/sec (whole node) {a.model} summarization fine-tune"
        base_batch, base = next(((bb, v) for (m, bb), v in HF_COMPARATOR_OTHER.items() if m == a.model),
                                (None, None))
    if env.is_main_process:
        print(json.dumps({
            "metric": metric,
            "value": round(value, 2), "unit": "samples/s", "n_gpus": n, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "mfu": round(mfu, 4), "tflops_per_gpu": round(step_flops / (ms * 1e-3) / n / 1e12, 1),
            "vs_baseline": round(value / (base * n), 3) if base and B >= 16 else None,
            "baseline_note": f"HF transformers+torch stack ({dtype_name}) measured on 1x MI355X at the same sequence "
                             f"shapes (its per-GPU batch {base_batch}, samples/s compared per sample) x N (BASELINE.md "
                             f"publishes no number)",
            "dtype": dtype_name, "data": "synthetic (random token ids, random-init weights)",
            "config": {"model": a.model, "global_batch": B * GA * n, "per_gpu_batch": B, "grad_accum": GA, "seq_len": S,
                       "target_len": T, "parallelism": f"dp{n}", "grad_ckpt": bool(a.grad_ckpt),
                       "bucket_mb": eng.reducer.bucket_sizes_mb()[1] if eng.reducer and len(eng.reducer.buckets) > 1 else None,
                       "tokens_per_s": round(value * (S + T), 1),
                       "grad_dtype": str(eng.flat.grad_buf.dtype).replace("torch.", ""),
                       "backend": env.backend, "world_size": n, "rccl_version": _rccl_version(),
                       "overlap": bool(eng.reducer.overlap) if eng.reducer else None,
                       "n_buckets": len(eng.reducer.buckets) if eng.reducer else None,
                       "comm_stress": bool(a.comm_stress), "hip_graph": graphed is not None,
                       "graph_error": graph_error,
                       "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)
                       if env.device.type == "cuda" else None},
            "comm": comm,
        }), flush=True)
    if n > 1:
        # orderly teardown: the native reducer holds the process group (and, on gloo, its worker threads): release it
        # before the group is destroyed, so nothing is torn down from interpreter-exit destructors
        _sync(env.device)
        if eng.reducer is not None:
            eng.reducer.remove()
            eng.reducer.native = None
        del eng, graphed
        import gc
        gc.collect()
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
