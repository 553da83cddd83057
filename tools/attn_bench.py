"""Microbenchmark of the attention kernels at T5/BART training shapes (fwd, bwd, TFLOP/s)."""
import argparse
import json
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd.ops import attention as A


def run(B, H, Sq, Sk, bias, kpm, causal, p, iters=20, sat=True):
    D = 64
    dev = "cuda"
    q = torch.randn(B, Sq, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Sk, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Sk, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    tab = torch.randn(32, H, device=dev, requires_grad=True) if bias else None
    mask = torch.ones(B, Sk, dtype=torch.bool, device=dev) if kpm else None
    lut = A.relative_bias_lut(tab, Sq, Sk, not causal, 32, 128) if bias else None
    if bias:  # sat=False: no saturated-bias ranges declared (every tile takes the LUT path)
        sat_r = lut._dllm_sat if sat else None
        lut = lut.detach()
        lut._dllm_sat = sat_r

    def fwd():
        return A.attention(q, k, v, scale=1.0, causal=causal, key_padding_mask=mask,
                           bias_lut=lut if bias else None, dropout_p=p, seed=1)
    o = fwd()
    g = torch.randn_like(o)
    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fwd()
    torch.cuda.synchronize()
    tf = (time.perf_counter() - t0) / iters
    lut2 = A.relative_bias_lut(tab, Sq, Sk, not causal, 32, 128) if bias else None
    if bias and not sat:
        lut2._dllm_sat = None
    def fb():
        o = A.attention(q, k, v, scale=1.0, causal=causal, key_padding_mask=mask, bias_lut=lut2, dropout_p=p, seed=1)
        o.backward(g, retain_graph=True)
    for _ in range(3):
        fb()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fb()
    torch.cuda.synchronize()
    tb = (time.perf_counter() - t0) / iters - tf
    fl = 4 * B * H * Sq * Sk * D * (0.5 if causal else 1.0)
    return {"B": B, "H": H, "Sq": Sq, "Sk": Sk, "bias": bias, "sat": bool(bias and sat), "kpm": kpm,
            "causal": causal, "p": p,
            "fwd_ms": tf * 1e3, "bwd_ms": tb * 1e3, "fwd_tflops": fl / tf / 1e12, "bwd_tflops": 2.5 * fl / tb / 1e12}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--ab", action="store_true", help="repeat every case 3x")
    a = ap.parse_args()
    cases = [(32, 12, 1024, 1024, True, True, False, 0.1), (32, 12, 1024, 1024, True, True, False, 0.0),
             (32, 12, 1024, 1024, False, False, False, 0.0), (32, 12, 128, 128, True, False, True, 0.1),
             (32, 12, 128, 1024, False, True, False, 0.1), (16, 16, 1024, 1024, False, True, False, 0.0)]
    if a.quick:
        cases = cases[:1]
    ap2 = a
    for c in cases:
        for rep in range(3 if ap2.ab else 1):
            print(json.dumps(run(*c)), flush=True)
