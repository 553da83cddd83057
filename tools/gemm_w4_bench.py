"""Projection GEMMs: one-wave-per-SIMD kernel (csrc/gemm_w4.hip) vs hipBLASLt (torch, shipped TunableOp table) vs the
8-wave ping-pong kernel (csrc/gemm_fused.hip variant 9) at every T5-base / BART-large linear-layer shape of one training
step at the bench batch (forward NT and input-gradient NN).  Rounds are interleaved in one process
(cdna_hip_programming.md §5.4 rule 24); the median over rounds is reported, on random operands.

    python tools/gemm_w4_bench.py [--iters 10] [--rounds 3] [--batch 256] [--grp 4]
    python tools/gemm_w4_bench.py --ablate --phases fwd --only "enc qkv"   # timing ablations of the w4 main loop

--ablate times the forward kernel with parts of its k-loop removed (csrc/gemm_w4.hip RS bits 4..7; results are
garbage, only the time counts): no DMAs, no fragment reads, no wait + barrier, no epilogue stores, and none of the
first three (MFMAs alone).
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd import _ext  # noqa: E402
from distributed_llms_example_amd.utils import tunableop  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def shapes(b):
    enc, dec, bl = 1024 * b, 128 * b, 1024 * (b // 8)
    return [("t5b enc qkv", enc, 768, 2304), ("t5b enc o", enc, 768, 768), ("t5b enc wi", enc, 768, 3072),
            ("t5b enc wo", enc, 3072, 768), ("t5b dec qkv", dec, 768, 2304), ("t5b dec o", dec, 768, 768),
            ("t5b dec wi", dec, 768, 3072), ("t5b dec wo", dec, 3072, 768), ("t5b cross kv", enc, 768, 18432),
            ("t5b lm head", dec, 768, 32128), ("bart enc qkv", bl, 1024, 3072), ("bart enc o", bl, 1024, 1024),
            ("bart enc fc2", bl, 4096, 1024)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--grp", type=int, default=4)
    ap.add_argument("--phases", default="fwd,dgrad")
    ap.add_argument("--only", default="")
    ap.add_argument("--ablate", action="store_true")
    a = ap.parse_args()
    tunableop.enable(0)
    C = _ext.native()
    for name, M, K, N in shapes(a.batch):
        if a.only and a.only not in name:
            continue
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        for phase in a.phases.split(","):
            if phase == "fwd":
                fl = 2.0 * M * K * N
                arms = {"lib": lambda: F.linear(x, w), "w4": lambda: C.gemm_w4(x, w, False, None, None, False, a.grp),
                        "w4np": lambda: C.gemm_w4(x, w, False, None, None, False, a.grp, False)}
                if C.gemm_fused_supported(x, w, False):
                    arms["pp9"] = lambda: C.gemm_fused(x, w, False, 0, None, None, None, 0.0, 0, 9)
            else:
                fl = 2.0 * M * K * N
                arms = {"lib": lambda: torch.matmul(dy, w), "w4": lambda: C.gemm_w4(dy, w, True, None, None, False, a.grp),
                        "w4np": lambda: C.gemm_w4(dy, w, True, None, None, False, a.grp, False)}
                if C.gemm_fused_supported(dy, w, True):
                    arms["pp9"] = lambda: C.gemm_fused(dy, w, True, 0, None, None, None, 0.0, 0, 9)
            ref = arms["lib"]().float()
            rec = {"shape": name, "phase": phase, "M": M, "K": K if phase == "fwd" else N, "N": N if phase == "fwd" else K}
            # the same call under other w4_sched values (csrc/gemm_w4.hip RS), set per arm below: "w4" / "w4np" run the
            # default; rs1 = the round-5 schedule
            # (769: + the early buffer release; 257: without it)
            rsv = {"w4": "769", "w4np": "769", "w4rs1": "1", "w4il": "257"}
            for k in ("w4rs1", "w4il"):
                arms[k] = arms["w4"]
            arms.pop("pp9", None)
            if a.ablate and phase == "fwd":
                for tag, v in (("nodma", "16"), ("noread", "32"), ("nobar", "64"), ("nostore", "128"),
                               ("mfmaonly", "112")):
                    arms["abl_" + tag] = arms["w4"]
                    rsv["abl_" + tag] = v
            for k, fn in arms.items():
                if k != "lib" and not k.startswith("abl_"):
                    os.environ["DLLM_ROUTE"] = "w4_sched=" + rsv.get(k, "769")
                    rec[f"{k}_relerr"] = float(f"{((fn().float() - ref).norm() / ref.norm()).item():.2e}")
            times = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, fn in arms.items():
                    os.environ["DLLM_ROUTE"] = "w4_sched=" + rsv.get(k, "769")
                    times[k].append(timeit(fn, a.iters))
            os.environ.pop("DLLM_ROUTE", None)
            for k, ts in times.items():
                t = statistics.median(ts)
                rec[f"{k}_us"] = round(t * 1e6, 1)
                rec[f"{k}_tflops"] = round(fl / t / 1e12, 1)
            print(json.dumps(rec), flush=True)
        del x, w, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
