import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from distributed_llms_example_amd.ops import attention as A

def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()

def case(B, H, Sq, Sk, bias, kpm, causal, p, scale):
    torch.manual_seed(0)
    D = 64; dev = "cuda"
    q = torch.randn(B, Sq, H, D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Sk, H, D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Sk, H, D, device=dev).to(torch.bfloat16)
    table = torch.randn(32, H, device=dev) * 0.5 if bias else None
    mask = None
    if kpm:
        mask = torch.ones(B, Sk, dtype=torch.bool, device=dev); mask[0, Sk - Sk // 5:] = False
    qs, ks, vs = (t.clone().requires_grad_(True) for t in (q, k, v))
    lut = A.relative_bias_lut(table, Sq, Sk, not causal, 32, 128, q_offset=Sk - Sq) if bias else None
    o = A.attention(qs, ks, vs, scale=scale, causal=causal, key_padding_mask=mask, bias_lut=lut, dropout_p=p, seed=7)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = A._reference(qr, kr, vr, scale, causal, mask, lut.float() if bias else None, p, 7)
    g = torch.randn_like(o)
    (o.float() * g.float()).sum().backward(); (ref * g.float()).sum().backward()
    dkerr = (ks.grad.float() - kr.grad).abs()
    bad = (dkerr > 1).nonzero()
    print(dict(B=B, Sq=Sq, Sk=Sk, bias=bias, kpm=kpm, p=p), "o", round(rel(o, ref), 4), "dq", round(rel(qs.grad, qr.grad), 4),
          "dk", rel(ks.grad, kr.grad), "dv", rel(vs.grad, vr.grad), "bad keys", bad[:, 1].unique()[:10].tolist(), flush=True)

for c in [(1, 1, 200, 200, False, False, False, 0.0, 1.0), (1, 1, 192, 200, False, False, False, 0.0, 1.0),
          (1, 1, 200, 200, True, False, False, 0.0, 1.0), (1, 1, 200, 200, False, True, False, 0.0, 1.0),
          (2, 3, 200, 200, True, True, False, 0.0, 1.0), (1, 1, 256, 256, False, False, False, 0.0, 1.0),
          (1, 1, 96, 96, False, False, False, 0.0, 1.0), (1, 1, 64, 64, False, False, False, 0.0, 1.0)]:
    case(*c)
