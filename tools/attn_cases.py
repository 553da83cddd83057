"""Fwd + bwd of one attention configuration, repeated (for rocprofv3 --kernel-trace --stats per-kernel times):
    python tools/attn_cases.py B H S bias kpm p scale [iters]
ATTN_SQ=n: n queries against the S keys (cross-attention; no bias)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd.ops import attention as A


def main():
    B, H, S = (int(x) for x in sys.argv[1:4])
    bias, kpm = sys.argv[4] == "1", sys.argv[5] == "1"
    p, scale = float(sys.argv[6]), float(sys.argv[7])
    iters = int(sys.argv[8]) if len(sys.argv) > 8 else 5
    D = 64
    torch.manual_seed(0)
    Sq = int(os.environ.get("ATTN_SQ", S))
    q = torch.randn(B, Sq, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(2))
    tab = torch.randn(32, H, device="cuda", requires_grad=True) if bias else None
    mask = torch.ones(B, S, dtype=torch.bool, device="cuda") if kpm else None
    g = None
    for it in range(iters):
        lut = A.relative_bias_lut(tab, S, S, True, 32, 128) if bias else None
        o = A.attention(q, k, v, scale=scale, key_padding_mask=mask, bias_lut=lut, dropout_p=p, seed=it)
        if g is None:
            g = torch.randn_like(o)
        o.backward(g)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
