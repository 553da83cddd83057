"""The LM-head GEMMs of one t5-base b=512 step (65536 decoder tokens x 32128 vocabulary x 768), each on hipBLASLt
(torch) and csrc/gemm_w4.hip: logits forward (NT), input gradient dH = dlogits W (NN, the 32128-deep reduction), weight
gradient dW = dlogitsᵀ H (w4 weight-gradient mode vs torch).  Interleaved rounds, median, random operands.

    python tools/lmhead_gemm_bench.py [--tokens 65536] [--vocab 32128] [--d 768] [--rounds 3]
"""
import argparse
import os
import statistics
import sys

import torch

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=32128)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    tunableop.enable(0)
    C = _ext.native()
    assert C is not None, _ext.load_error()
    N, V, d = a.tokens, a.vocab, a.d
    h = torch.randn(N, d, device="cuda").to(torch.bfloat16)
    w = (torch.randn(V, d, device="cuda") * d ** -0.5).to(torch.bfloat16)
    g = (torch.randn(N, V, device="cuda") * 1e-3).to(torch.bfloat16)
    gw32 = torch.zeros(V, d, device="cuda", dtype=torch.float32)
    fl = 2.0 * N * V * d
    cases = {
        "fwd logits  lib": lambda: torch.mm(h, w.t()),
        "fwd logits  w4": lambda: C.gemm_w4(h, w, False),
        "dgrad dH    lib": lambda: torch.mm(g, w),
        "dgrad dH    w4": lambda: C.gemm_w4(g, w, True),
        "wgrad dW    lib": lambda: gw32.add_(torch.mm(g.t(), h, out_dtype=torch.float32)),
        "wgrad dW    w4": lambda: C.gemm_wgrad(g, h, gw32, True, -1, 0),
    }
    # agreement of the two arms (dH: relative Frobenius error vs the fp32 product)
    ref = (g[:4096].float() @ w.float())
    got = C.gemm_w4(g[:4096].contiguous(), w, True).float()
    print(f"# dgrad w4 vs fp32 (4096 rows): rel err {((got - ref).norm() / ref.norm()).item():.2e}", flush=True)
    ts = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, fn in cases.items():
            ts[k].append(timeit(fn, a.iters))
    print(f"# LM head GEMMs, {N} tokens x {V} vocab x {d}: {fl / 1e12:.2f} TFLOP each; median of {a.rounds} rounds")
    for k, t in ts.items():
        m = statistics.median(t)
        print(f"{k:18s} {m * 1e3:8.3f} ms  {fl / m / 1e12:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
