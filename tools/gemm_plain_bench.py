"""Projection GEMMs without epilogue: hipBLASLt (torch, shipped TunableOp table) vs csrc/gemm_fused.hip (epi 0) at
every T5-base / BART-large linear-layer shape of one training step (forward NT and input-gradient NN).

    python tools/gemm_plain_bench.py [--iters 20] [--variants 0,3]
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
    ap.add_argument("--phases", default="fwd,dgrad")
    a = ap.parse_args()
    tunableop.enable(0)
    C = _ext.native()
    # a variant "8g4" runs variant 8 with DLLM_ROUTE gemm_grp=4 (tile-order group size, read per call by the binding)
    variants = a.variants.split(",")
    # (name, tokens M, in K, out N): t5-base at b=64 (enc 65536 tokens, dec 8192), bart-large at b=32
    shapes = [("t5b enc qkv", 65536, 768, 2304), ("t5b enc o", 65536, 768, 768), ("t5b enc wi", 65536, 768, 3072),
              ("t5b enc wo", 65536, 3072, 768), ("t5b dec qkv", 8192, 768, 2304), ("t5b dec o", 8192, 768, 768),
              ("t5b dec wi", 8192, 768, 3072), ("t5b dec wo", 8192, 3072, 768), ("t5b cross kv", 65536, 768, 18432),
              ("bart enc qkv", 32768, 1024, 3072), ("bart enc o", 32768, 1024, 1024),
              ("bart enc fc2", 32768, 4096, 1024)]
    for name, M, K, N in shapes:
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        fl = 2.0 * M * K * N
        for phase in a.phases.split(","):
            rec = {"shape": name, "phase": phase, "M": M, "K": K if phase == "fwd" else N, "N": N if phase == "fwd" else K}
            if phase == "fwd":
                lib = lambda: F.linear(x, w)  # noqa: E731
                mk = lambda v: (lambda: C.gemm_fused(x, w, False, 0, None, None, None, 0.0, 0, v))  # noqa: E731
                ok = C.gemm_fused_supported(x, w, False)
            else:
                lib = lambda: torch.matmul(dy, w)  # noqa: E731
                mk = lambda v: (lambda: C.gemm_fused(dy, w, True, 0, None, None, None, 0.0, 0, v))  # noqa: E731
                ok = C.gemm_fused_supported(dy, w, True)
            ref = lib().float()
            t = timeit(lib, a.iters)
            rec["lib_us"] = round(t * 1e6, 1)
            rec["lib_tflops"] = round(fl / t / 1e12, 1)
            if ok:
                for vi, v in enumerate(variants):
                    tag = f"v{v}" + ("b" * variants[:vi].count(v))  # a repeated variant (A/B/A order) gets its own key
                    vv, _, grp = v.partition("g")
                    os.environ["DLLM_ROUTE"] = f"gemm_grp={grp or 0}"
                    fn = mk(int(vv))
                    out = fn().float()
                    rec[f"{tag}_relerr"] = float(f"{((out - ref).norm() / ref.norm()).item():.2e}")
                    t = timeit(fn, a.iters)
                    rec[f"{tag}_us"] = round(t * 1e6, 1)
                    rec[f"{tag}_tflops"] = round(fl / t / 1e12, 1)
            print(json.dumps(rec), flush=True)
        del x, w, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
