"""Per-feature anatomy of the attention kernels: runs fwd + bwd of the T5 encoder self-attention shape under several
feature sets (relative-bias LUT b, key-padding mask k, dropout d), so a kernel trace (rocprofv3 --kernel-trace --stats)
prices each feature by the template instance it selects.  Each config is a string like "b1k1d1"; --nosat declares no
saturated-bias ranges (every tile takes the LUT path)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd.ops import attention as A


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--S", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cfg", default="b1k1d1,b0k1d1,b1k1d0,b0k0d0")
    ap.add_argument("--nosat", action="store_true")
    a = ap.parse_args()
    B, H, S, D = a.B, a.H, a.S, 64
    dev = "cuda"
    torch.manual_seed(0)
    q = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    tab = torch.randn(32, H, device=dev, requires_grad=True)
    for cfg in a.cfg.split(","):
        bias, kpm, drop = cfg[1] == "1", cfg[3] == "1", cfg[5] == "1"
        mask = torch.ones(B, S, dtype=torch.bool, device=dev) if kpm else None
        g = None
        for it in range(a.iters + 2):
            lut = A.relative_bias_lut(tab, S, S, True, 32, 128) if bias else None
            if bias and a.nosat:
                lut._dllm_sat = None
            o = A.attention(q, k, v, scale=1.0, key_padding_mask=mask, bias_lut=lut, dropout_p=0.1 if drop else 0.0,
                            seed=it)
            if g is None:
                g = torch.randn_like(o)
            o.backward(g)
        torch.cuda.synchronize()
        print(cfg, "done", flush=True)


if __name__ == "__main__":
    main()
