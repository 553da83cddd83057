"""Forward-only attention check vs the fp32 reference over a grid of small cases (NaN / error localisation)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llms_example_amd.ops import attention as A  # noqa: E402


def case(B, H, Sq, Sk, bias, kpm, causal, p, scale):
    torch.manual_seed(0)
    D, dev = 64, "cuda"
    q = torch.randn(B, Sq, H, D, device=dev).to(torch.bfloat16)
    k = torch.randn(B, Sk, H, D, device=dev).to(torch.bfloat16)
    v = torch.randn(B, Sk, H, D, device=dev).to(torch.bfloat16)
    table = torch.randn(32, H, device=dev) * 0.5 if bias else None
    mask = None
    if kpm:
        mask = torch.ones(B, Sk, dtype=torch.bool, device=dev)
        mask[0, Sk - Sk // 5:] = False
    lut = A.relative_bias_lut(table, Sq, Sk, not causal, 32, 128, q_offset=Sk - Sq) if bias else None
    o = A.attention(q, k, v, scale=scale, causal=causal, key_padding_mask=mask, bias_lut=lut, dropout_p=p, seed=7)
    ref = A._reference(q.float(), k.float(), v.float(), scale, causal, mask, lut.float() if bias else None, p, 7)
    err = (o.float() - ref).abs()
    nan = torch.isnan(o.float())
    rows = nan.any(-1).any(-1).nonzero()[:, 1].unique().tolist() if nan.any() else []
    print(dict(B=B, H=H, Sq=Sq, Sk=Sk, bias=bias, kpm=kpm, causal=causal, p=p),
          "rel", round(((o.float() - ref).norm() / ref.norm()).item(), 5), "maxerr", round(err.nan_to_num(9).max().item(), 4),
          "nan rows", rows[:20], flush=True)


for c in [(2, 2, 96, 96, False, False, True, 0.0, 0.125), (2, 2, 96, 96, False, False, True, 0.1, 0.125),
          (2, 2, 96, 96, False, False, False, 0.1, 0.125), (2, 2, 256, 256, False, False, False, 0.1, 0.125),
          (2, 2, 256, 256, True, True, False, 0.1, 1.0), (2, 2, 256, 256, True, False, True, 0.1, 1.0),
          (2, 2, 128, 128, False, False, True, 0.1, 0.125), (1, 1, 64, 64, False, False, True, 0.1, 0.125)]:
    case(*c)
