"""Weight-gradient GEMMs at micro-batch token counts: csrc/gemm_w4.hip's weight-gradient mode (auto split count) vs
hipBLASLt (torch.addmm into the fp32 gradient, bf16 operands) at the t5-base layer shapes, for the token counts of the
reference's micro-batches (b=1: 1024 encoder / 128 decoder rows; b=8: 8192 / 1024).  Interleaved rounds, median.

    python tools/wgrad_small_bench.py [--iters 50] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd import _ext  # noqa: E402
from distributed_llms_example_amd.utils import tunableop  # noqa: E402


def timeit(fn, iters):
    """GPU time per call: `iters` calls captured in one HIP graph and replayed (no host launch cost, as in a graphed
    training step)."""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * iters) * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    tunableop.enable(0)
    C = _ext.native()
    assert C is not None, "native library not loaded"
    # (name, out features M, in features N): dW [M, N] = dY[K, M]^T X[K, N]
    layers = [("qkv", 2304, 768), ("o", 768, 768), ("wi", 3072, 768), ("wo", 768, 3072), ("cross kv", 1536, 768)]
    for K in (128, 1024, 2048, 4096, 8192, 16384):
        for name, M, N in layers:
            dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)
            x = torch.randn(K, N, device="cuda").to(torch.bfloat16)
            g = torch.zeros(M, N, device="cuda", dtype=torch.float32)
            arms = {"w4": lambda: C.gemm_wgrad(dy, x, g, True, -1, 0),
                    "lib": lambda: torch.addmm(g, dy.t(), x, out_dtype=torch.float32, out=g)}
            ref = (dy.double().t() @ x.double()).float()
            rec = {"K": K, "layer": name, "M": M, "N": N}
            for k, fn in arms.items():
                g.zero_()
                fn()
                rec[f"{k}_relerr"] = float(f"{((g - ref).norm() / ref.norm()).item():.2e}")
            times = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, fn in arms.items():
                    times[k].append(timeit(fn, a.iters))
            for k, ts in times.items():
                rec[f"{k}_us"] = round(statistics.median(ts) * 1e6, 1)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
