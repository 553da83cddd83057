"""FFN GEMM-with-epilogue microbenchmark: csrc/gemm_fused.hip variants vs hipBLASLt (+ the separate activation
kernel of csrc/act.hip) at the T5-base / BART-large FFN shapes (tokens = batch x seq), bf16, random data.

Forward   wi:  H = dropout(act(X Wiᵀ))        library: F.linear + act_fwd kernel
Backward  wo:  dU = act'(dropout'(dY Wo))      library: matmul + act_bwd kernel

    python tools/gemm_fused_bench.py [--iters 20] [--variants 0,1,2,3]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd import _ext  # noqa: E402
from distributed_llms_example_amd.utils import tunableop  # noqa: E402

EPI = {"relu": (1, 3, 0), "gelu": (2, 4, 1)}  # act -> (fwd epilogue, bwd epilogue, csrc/act.hip act id)


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default="3,4")
    ap.add_argument("--p", type=float, default=0.1)
    a = ap.parse_args()
    tunableop.enable(0)
    C = _ext.native()
    variants = [int(v) for v in a.variants.split(",")]
    # (tokens, d_model, d_ff, act): t5-base encoder / decoder at b=64, bart-large encoder at b=32, t5-large
    shapes = [(65536, 768, 3072, "relu"), (8192, 768, 3072, "relu"), (32768, 1024, 4096, "gelu"),
              (16384, 1024, 4096, "relu")]
    for M, d, Fd, act in shapes:
        efwd, ebwd, aid = EPI[act]
        p = a.p if act == "relu" else 0.0
        x = torch.randn(M, d, device="cuda").to(torch.bfloat16)
        wi = (torch.randn(Fd, d, device="cuda") * d ** -0.5).to(torch.bfloat16)
        wo = (torch.randn(d, Fd, device="cuda") * Fd ** -0.5).to(torch.bfloat16)
        dy = torch.randn(M, d, device="cuda").to(torch.bfloat16)
        fl = 2.0 * M * d * Fd
        u_pre = F.linear(x, wi)
        h_act = C.act_fwd(u_pre, aid, False, p, 7)
        for phase in ("fwd", "bwd"):
            rec = {"phase": phase, "M": M, "d": d, "F": Fd, "act": act, "p": p}
            if phase == "fwd":
                def lib():
                    return C.act_fwd(F.linear(x, wi), aid, False, p, 7)
                aux = torch.empty(M, Fd, device="cuda", dtype=torch.bfloat16) if efwd == 2 else None

                def mk(v):
                    return lambda: C.gemm_fused(x, wi, False, efwd, None, None, aux, p, 7, v)
            else:
                aux_b = h_act if ebwd == 3 else u_pre

                def lib():
                    return C.act_bwd(torch.matmul(dy, wo), u_pre, aid, False, p, 7)

                def mk(v):
                    return lambda: C.gemm_fused(dy, wo, True, ebwd, None, aux_b, None, p, 7, v)
            ref = lib().float()
            t = timeit(lib, a.iters)
            rec["lib_us"] = round(t * 1e6, 1)
            rec["lib_tflops"] = round(fl / t / 1e12, 1)
            for vi, v in enumerate(variants):
                tag = f"v{v}" + ("b" * variants[:vi].count(v))  # a repeated variant (A/B/A order) gets its own key
                fn = mk(v)
                out = fn().float()
                rec[f"{tag}_relerr"] = float(f"{((out - ref).norm() / ref.norm()).item():.2e}")
                t = timeit(fn, a.iters)
                rec[f"{tag}_us"] = round(t * 1e6, 1)
                rec[f"{tag}_tflops"] = round(fl / t / 1e12, 1)
            print(json.dumps(rec), flush=True)
        del x, wi, wo, dy, u_pre, h_act
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
