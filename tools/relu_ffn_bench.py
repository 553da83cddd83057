"""T5 ReLU FFN GEMMs at the t5-base encoder shape: the forward with ReLU + dropout + keep/positive bit mask (ping-pong
csrc/gemm_fused.hip epilogue 1 vs csrc/gemm_w4.hip W4_EPI_RELU, with and without the dropout hash) and the backward
through the mask (w4 W4_EPI_DRELU_M), against the same GEMMs without epilogue (w4 plain, hipBLASLt).

    python tools/relu_ffn_bench.py --rounds 5
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd import _ext  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--M", type=int, default=524288)
    a = ap.parse_args()
    C = _ext.native()
    dev = "cuda"
    M, d, F = a.M, 768, 3072
    x = torch.randn(M, d, device=dev).to(torch.bfloat16)
    wi = (torch.randn(F, d, device=dev) * d ** -0.5).to(torch.bfloat16)
    wo = (torch.randn(d, F, device=dev) * F ** -0.5).to(torch.bfloat16)
    dy = torch.randn(M, d, device=dev).to(torch.bfloat16)
    mask_pp = torch.empty(M * F // 32, device=dev, dtype=torch.int32)
    mask_w4 = torch.empty(C.gemm_w4_mask_words(M, F), device=dev, dtype=torch.int32)
    C.gemm_fused(x, wi, False, 1, None, None, None, 0.1, 1, -1, mask_pp)
    arms = {
        "pp_relu_drop_fwd": lambda: C.gemm_fused(x, wi, False, 1, None, None, None, 0.1, 1, -1, mask_pp),
        "w4_relu_drop_fwd": lambda: C.gemm_w4(x, wi, False, None, None, False, -1, True, 1, 0.1, 1, mask_w4),
        "w4_relu_nodrop_fwd": lambda: C.gemm_w4(x, wi, False, None, None, False, -1, True, 1, 0.0, 1, mask_w4),
        "w4_relu_drop_fwd_np": lambda: C.gemm_w4(x, wi, False, None, None, False, -1, False, 1, 0.1, 1, mask_w4),
        "w4_plain_fwd_np": lambda: C.gemm_w4(x, wi, False, None, None, False, -1, False),
        "w4_plain_fwd": lambda: C.gemm_w4(x, wi, False),
        "lib_fwd": lambda: torch.nn.functional.linear(x, wi),
        "w4_drelu_bwd": lambda: C.gemm_w4(dy, wo, True, None, None, False, -1, True, 7, 0.1, 1, mask_pp, True),
        "w4_plain_bwd": lambda: C.gemm_w4(dy, wo, True),
        "lib_bwd": lambda: torch.matmul(dy, wo),
    }
    t = {k: [] for k in arms}
    for _ in range(a.rounds):
        for k, fn in arms.items():
            t[k].append(timeit(fn, a.iters))
    fl = 2.0 * M * d * F
    print(json.dumps({"M": M, "d": d, "F": F, **{k: {"us": round(statistics.median(v), 1),
                                                      "tflops": round(fl / statistics.median(v) / 1e6, 1)}
                                                  for k, v in t.items()}}), flush=True)


if __name__ == "__main__":
    main()
