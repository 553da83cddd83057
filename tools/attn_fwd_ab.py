"""Attention forward A/B in one process: kernel variants selected per call by an environment variable (e.g.
DLLM_ATTN_FWD_PIPE=0/1), interleaved over rounds at training shapes, median ms and TFLOP/s per arm.

    python tools/attn_fwd_ab.py --env DLLM_ATTN_FWD_PIPE --arms 0,1 --rounds 5
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd.ops import attention as A  # noqa: E402

# name: (B, H, Sq, Sk, T5 bias, key padding, causal, dropout)
CASES = {
    "t5-base enc": (128, 12, 1024, 1024, True, True, False, 0.1),
    "t5-base dec self": (128, 12, 128, 128, True, False, True, 0.1),
    "t5-base cross": (128, 12, 128, 1024, False, True, False, 0.1),
    "bart enc": (64, 16, 1024, 1024, False, True, False, 0.0),
    "bart dec causal 1024": (64, 16, 1024, 1024, False, False, True, 0.0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="DLLM_ATTN_FWD_PIPE")
    ap.add_argument("--arms", default="0,1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cases", default=None, help="comma list of case names (default all)")
    a = ap.parse_args()
    dev = "cuda"
    names = a.cases.split(",") if a.cases else list(CASES)
    arms = a.arms.split(",")
    for name in names:
        B, H, Sq, Sk, bias, kpm, causal, p = CASES[name]
        q = torch.randn(B, Sq, H, 64, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, Sk, H, 64, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, Sk, H, 64, device=dev, dtype=torch.bfloat16)
        lut = None
        if bias:
            lut = A.relative_bias_lut(torch.randn(32, H, device=dev) * 0.5, Sq, Sk, not causal, 32, 128)
        mask = None
        if kpm:
            mask = torch.ones(B, Sk, dtype=torch.bool, device=dev)
            mask[::3, Sk - Sk // 7:] = False
        flops = 4 * B * H * Sq * Sk * 64 * (0.5 if causal and Sq == Sk else 1.0)

        def fwd():
            return A.attention(q, k, v, scale=1.0, causal=causal, key_padding_mask=mask, bias_lut=lut, dropout_p=p,
                               seed=11)

        times = {arm: [] for arm in arms}
        for _ in range(a.rounds):
            for arm in arms:
                os.environ[a.env] = arm
                fwd()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    fwd()
                torch.cuda.synchronize()
                times[arm].append((time.perf_counter() - t0) / a.iters * 1e3)
        out = {"case": name, "env": a.env}
        for arm in arms:
            med = statistics.median(times[arm])
            out[arm] = {"ms": round(med, 4), "tflops": round(flops / med / 1e9, 1), "min_ms": round(min(times[arm]), 4)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
