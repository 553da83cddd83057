"""fp32 flash attention (csrc/attn_f32.hip) against an fp64 torch reference of the same op: forward output, dQ/dK/dV
and the bias-LUT gradient, with the T5 bias, key padding, causal masks, BART scaling and attention dropout (the exact
keep decisions of ops/rng.py attention_keep_mask), on ragged lengths that are not multiples of the 64-row tiles."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref64(q, k, v, scale, causal, kpm, lut, p, seed):
    """fp64 reference: scores, bias, masks, softmax, dropout (same keep bits), probabilities @ V."""
    from distributed_llms_example_amd.ops.rng import attention_keep_mask
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    qf, kf, vf = (t.double().permute(0, 2, 1, 3) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if lut is not None:
        rel = torch.arange(Sk, device=q.device)[None, :] - torch.arange(Sq, device=q.device)[:, None] + (Sq - 1)
        s = s + lut.double()[:, rel].unsqueeze(0)
    neg = torch.finfo(torch.float64).min
    if kpm is not None:
        s = s.masked_fill(~kpm.bool()[:, None, None, :], neg)
    if causal:
        cm = torch.arange(Sk, device=q.device)[None, :] > (torch.arange(Sq, device=q.device)[:, None] + Sk - Sq)
        s = s.masked_fill(cm, neg)
    pr = torch.softmax(s, dim=-1)
    if p > 0.0:
        keep = attention_keep_mask(seed, p, B, H, Sq, Sk, q.device)
        pr = pr * keep.double() / (1.0 - p)
    return torch.matmul(pr, vf).permute(0, 2, 1, 3)


CASES = [
    # B, Sq, Sk, H, scale, causal, kpm, bias, p
    (2, 200, 200, 3, 1.0, False, True, True, 0.1),     # T5 encoder self-attention
    (2, 130, 130, 2, 1.0, True, False, True, 0.1),     # T5 decoder self-attention (causal + bias)
    (2, 70, 190, 2, 0.125, False, True, False, 0.0),   # BART cross-attention
    (1, 64, 128, 2, 0.125, True, False, False, 0.0),   # causal with Sk > Sq
    (3, 96, 96, 2, 1.0, False, False, True, 0.0),
]


@pytest.mark.parametrize("B,Sq,Sk,H,scale,causal,use_kpm,bias,p", CASES)
def test_attn_f32_matches_fp64(B, Sq, Sk, H, scale, causal, use_kpm, bias, p):
    from distributed_llms_example_amd import _ext
    from distributed_llms_example_amd.ops.attention import attention
    assert _ext.native() is not None
    torch.manual_seed(0)
    dev = "cuda"
    q = torch.randn(B, Sq, H, 64, device=dev, requires_grad=True)
    k = torch.randn(B, Sk, H, 64, device=dev, requires_grad=True)
    v = torch.randn(B, Sk, H, 64, device=dev, requires_grad=True)
    kpm = None
    if use_kpm:
        kpm = torch.ones(B, Sk, dtype=torch.bool, device=dev)
        kpm[0, -37:] = False
    lut = (torch.randn(H, Sq + Sk - 1, device=dev) * 0.5).requires_grad_(True) if bias else None
    seed = 1234
    o = attention(q, k, v, scale=scale, causal=causal, key_padding_mask=kpm, bias_lut=lut, dropout_p=p, seed=seed)
    assert o.dtype == torch.float32
    g = torch.randn_like(o)
    grads = torch.autograd.grad(o, [q, k, v] + ([lut] if bias else []), g)

    q64, k64, v64 = (t.detach().double().requires_grad_(True) for t in (q, k, v))
    lut64 = lut.detach().double().requires_grad_(True) if bias else None
    o64 = _ref64(q64, k64, v64, scale, causal, kpm, lut64, p, seed)
    grads64 = torch.autograd.grad(o64, [q64, k64, v64] + ([lut64] if bias else []), g.double())

    def rel(a, b):
        return ((a.double() - b).norm() / b.norm().clamp_min(1e-30)).item()

    assert rel(o, o64) < 2e-6, rel(o, o64)
    for name, a, b in zip(["dq", "dk", "dv", "dlut"], grads, grads64):
        assert rel(a, b) < 2e-5, (name, rel(a, b))


def test_attn_f32_kernel_runs_not_composite(monkeypatch):
    """fp32 attention on the GPU goes to csrc/attn_f32.hip (the O(S^2) composite only with routing attn_f32=0)."""
    from distributed_llms_example_amd import _ext
    from distributed_llms_example_amd.ops import attention as A
    calls = []
    real = _ext.native().attn_f32_fwd

    class Spy:
        def __getattr__(self, n):
            if n == "attn_f32_fwd":
                def f(*a, **kw):
                    calls.append(1)
                    return real(*a, **kw)
                return f
            return getattr(_ext.native(), n)

    monkeypatch.setattr(A._ext, "native", lambda: Spy())
    x = torch.randn(1, 64, 2, 64, device="cuda")
    A.attention(x, x, x)
    assert calls == [1]
