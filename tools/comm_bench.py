#!/usr/bin/env python
"""All-reduce microbenchmark for gradient-bucket sizing.

rccl-tests binaries are not shipped in this image, so this measures what the reducer actually issues:
``torch.distributed.all_reduce`` (RCCL over xGMI under the "nccl" backend) on contiguous bf16 slices of one
flat buffer, AVG, for a sweep of bucket sizes.  Bus bandwidth = algbw * 2 (N-1) / N (ring convention).

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 tools/comm_bench.py
    DLLM_FORCE_CPU=1 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        tools/comm_bench.py --sizes-mb 1,4 --iters 3          # gloo rehearsal on CPU

Sweep mode (a driver process, no collective of its own): RCCL reads NCCL_ALGO / NCCL_PROTO / NCCL_MIN_NCHANNELS
when the communicator is created, so every setting is a fresh ``torch.distributed.run`` child; their JSON lines are
collected into one summary (per size: the best setting and its bus bandwidth), ready for the first 8-GPU lease:

    python tools/comm_bench.py --sweep --nproc 8 --algos default,Ring,Tree --channels 0,16,32 \\
        --sizes-mb 1,16,64,128,256 --out gpurun_out/comm_sweep.json
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


def sweep(a):
    """Run one torchrun child per (algo, proto, min-channels) setting and summarise."""
    import itertools
    import subprocess
    rows = []
    port = a.port
    for algo, proto, ch in itertools.product(a.algos.split(","), a.protos.split(","), a.channels.split(",")):
        env = dict(os.environ)
        for k, v in (("NCCL_ALGO", algo), ("NCCL_PROTO", proto)):
            if v and v != "default":
                env[k] = v
            else:
                env.pop(k, None)
        if ch and ch != "0":
            env["NCCL_MIN_NCHANNELS"] = ch
        else:
            env.pop("NCCL_MIN_NCHANNELS", None)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.nproc}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__),
               "--sizes-mb", a.sizes_mb, "--iters", str(a.iters), "--warmup", str(a.warmup), "--dtype", a.dtype]
        port += 1
        setting = {"algo": algo, "proto": proto, "min_nchannels": int(ch or 0)}
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=a.child_timeout)
        ok = 0
        for line in r.stdout.splitlines():
            if line.startswith("{") and '"busbw_GBps"' in line:
                rec = json.loads(line)
                rec.update(setting)
                rows.append(rec)
                ok += 1
                print(json.dumps(rec), flush=True)
        if r.returncode != 0 or ok == 0:
            print(json.dumps({**setting, "error": f"rc={r.returncode}", "tail": r.stdout[-400:]}), flush=True)
    best = {}
    for rec in rows:
        k = rec["size_mb"]
        if k not in best or rec["busbw_GBps"] > best[k]["busbw_GBps"]:
            best[k] = rec
    summary = {"nproc": a.nproc, "dtype": a.dtype, "runs": rows,
               "best": [{"size_mb": k, "busbw_GBps": v["busbw_GBps"], "us": v["us"], "algo": v["algo"],
                         "proto": v["proto"], "min_nchannels": v["min_nchannels"]} for k, v in sorted(best.items())]}
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(summary, f, indent=1)
    print(json.dumps({"best": summary["best"]}), flush=True)
    return summary


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="1,4,16,32,64,128,256,512")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--sweep", action="store_true", help="driver: one torchrun child per RCCL setting")
    ap.add_argument("--nproc", type=int, default=8)
    ap.add_argument("--algos", default="default,Ring,Tree")
    ap.add_argument("--protos", default="default")
    ap.add_argument("--channels", default="0,16,32")
    ap.add_argument("--port", type=int, default=29610)
    ap.add_argument("--child-timeout", type=float, default=600.0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.sweep:
        sweep(a)
        return
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
