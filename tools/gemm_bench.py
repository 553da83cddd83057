"""Weight-gradient GEMM microbenchmark: csrc/gemm.hip variants vs torch (hipBLASLt + TunableOp table)
at the T5-base / BART-large training shapes (tokens = batch x seq)."""
import argparse
import json
import os
import sys
import time

import torch

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
    ap.add_argument("--variants", default="0,4,9")
    ap.add_argument("--shapes", default=None, help="K:M:N,... (default: the T5/BART training set)")
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--c-f32", action="store_true", help="fp32 output (the fp32 flat gradient buffer)")
    a = ap.parse_args()
    tunableop.enable(0)
    C = _ext.native()
    shapes = [(65536, 768, 768), (65536, 2304, 768), (65536, 3072, 768), (65536, 768, 3072),
              (65536, 18432, 768), (8192, 768, 768), (8192, 2304, 768), (8192, 3072, 768), (8192, 768, 3072),
              (32768, 1024, 1024), (32768, 4096, 1024), (32768, 1024, 4096)]
    if a.shapes:
        shapes = [tuple(int(x) for x in sh.split(":")) for sh in a.shapes.split(",")]
    for K, M, N in shapes:
        dy = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(M, N, device="cuda", dtype=torch.float32 if a.c_f32 else torch.bfloat16)
        fl = 2.0 * K * M * N
        rec = {"K": K, "M": M, "N": N}
        if not a.no_torch:
            t = timeit(lambda: g.addmm_(dy.t(), x), a.iters)
            rec["torch_us"] = round(t * 1e6, 1)
            rec["torch_tflops"] = round(fl / t / 1e12, 1)
        ref = dy.float().t() @ x.float()
        vs = list(map(int, a.variants.split(",")))
        for vi, v in enumerate(vs):
            tag = f"v{v}" + ("b" * vs[:vi].count(v))  # repeated variants (A/B/A order) get their own keys
            g.zero_()
            C.gemm_wgrad(dy, x, g, True, v, 0)
            err = ((g.float() - ref).norm() / ref.norm()).item()
            t = timeit(lambda: C.gemm_wgrad(dy, x, g, True, v, 0), a.iters)
            rec[f"{tag}_us"] = round(t * 1e6, 1)
            rec[f"{tag}_tflops"] = round(fl / t / 1e12, 1)
            rec[f"{tag}_relerr"] = float(f"{err:.2e}")
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
