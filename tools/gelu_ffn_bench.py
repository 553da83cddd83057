"""GELU FFN GEMMs: the ping-pong kernel's epilogues 2 / 4 (csrc/gemm_fused.hip) vs the w4 kernel's GELU epilogues
(csrc/gemm_w4.hip W4_EPI_GELU / W4_EPI_DGELU) at BART shapes, interleaved rounds, median us and TF/s.

    python tools/gelu_ffn_bench.py --rounds 5
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
    a = ap.parse_args()
    C = _ext.native()
    dev = "cuda"
    for M, d, F in ((262144, 1024, 4096), (32768, 1024, 4096)):
        x = torch.randn(M, d, device=dev).to(torch.bfloat16)
        wi = (torch.randn(F, d, device=dev) * d ** -0.5).to(torch.bfloat16)
        bi = torch.randn(F, device=dev).to(torch.bfloat16)
        wo = (torch.randn(d, F, device=dev) * F ** -0.5).to(torch.bfloat16)
        dy = torch.randn(M, d, device=dev).to(torch.bfloat16)
        aux = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
        part = torch.empty(M // 128, F, device=dev)
        arms = {
            "pp_fwd": lambda: C.gemm_fused(x, wi, False, 2, bi, None, aux, 0.0, 1, -1),
            "w4_fwd": lambda: C.gemm_w4(x, wi, False, bi, None, False, -1, True, 11, 0.0, 1, None, False, None, aux),
            "pp_bwd": lambda: C.gemm_fused(dy, wo, True, 4, None, aux, None, 0.0, 1, -1, None, part),
            "w4_bwd": lambda: C.gemm_w4(dy, wo, True, None, None, False, -1, False, 12, 0.0, 0, None, False, aux, None,
                                        part),
            "w4_plain_fwd": lambda: C.gemm_w4(x, wi, False, bi),
            "lib_fwd": lambda: torch.nn.functional.linear(x, wi, bi),
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
