#!/usr/bin/env python
"""All-reduce microbenchmark for gradient-bucket sizing.

rccl-tests binaries are not shipped in this image, so this measures what the reducer actually issues:
``torch.distributed.all_reduce`` (RCCL over xGMI under the "nccl" backend) on contiguous bf16 slices of one
flat buffer, AVG, for a sweep of bucket sizes.  Bus bandwidth = algbw * 2 (N-1) / N (ring convention).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 tools/comm_bench.py
    DLLM_FORCE_CPU=1 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        tools/comm_bench.py --sizes-mb 1,4 --iters 3          # gloo rehearsal on CPU
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd.parallel.env import init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,32,64,128,256,512")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    env = init_distributed()
    n = env.world_size
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    esz = torch.tensor([], dtype=dt).element_size()
    sizes = [float(s) for s in a.sizes_mb.split(",")]
    buf = torch.ones(int(max(sizes) * 2**20 // esz), dtype=dt, device=env.device)
    op = dist.ReduceOp.AVG if env.backend == "nccl" else dist.ReduceOp.SUM

    def sync():
        if env.device.type == "cuda":
            torch.cuda.synchronize()

    for mb in sizes:
        view = buf[: int(mb * 2**20 // esz)]
        for _ in range(a.warmup):
            dist.all_reduce(view, op=op)
        sync()
        env.barrier()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            dist.all_reduce(view, op=op)
        sync()
        dt_s = (time.perf_counter() - t0) / a.iters
        t = torch.tensor([dt_s], dtype=torch.float64, device=env.device if env.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt_s = t.item()
        algbw = view.numel() * esz / dt_s / 1e9
        if env.is_main_process:
            print(json.dumps({"bytes": view.numel() * esz, "size_mb": mb, "n": n, "backend": env.backend,
                              "us": round(dt_s * 1e6, 1), "algbw_GBps": round(algbw, 2),
                              "busbw_GBps": round(algbw * 2 * (n - 1) / n, 2)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
