"""HIP kernel numerics vs plain-PyTorch fp32 references (SURVEY.md §4 level 1).

Every test runs the native (gfx950) op on bf16 inputs and the reference implementation of the SAME
op in fp32 on the same (bf16-rounded) values; dropout uses the shared counter-based mask so p > 0
is compared exactly, not statistically.  Also asserts the native extension is the code that ran.
"""
import math

import pytest
import torch

from distributed_llms_example_amd import _ext
from distributed_llms_example_amd.ops import activations, attention as A, cross_entropy as CE, norms

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, rtol, atol, msg=""):
    a = a.float()
    b = b.float()
    err = (a - b).abs()
    lim = atol + rtol * b.abs()
    bad = (err > lim).float().mean().item()
    assert bad < 1e-3, f"{msg}: {bad*100:.3f}% elements out of tol; max err {err.max().item():.4g}"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def test_native_extension_loaded():
    assert _ext.native() is not None, _ext.load_error()
    assert _ext.native().arch == "gfx950"
    x = torch.randn(8, 64, device=DEV, dtype=torch.bfloat16)
    assert _ext.use_native(x)


@pytest.mark.parametrize("kind", [norms.RMS, norms.LAYER])
@pytest.mark.parametrize("d", [64, 512, 768, 1024, 2048])
@pytest.mark.parametrize("resid,p", [(False, 0.0), (True, 0.0), (True, 0.1), (False, 0.1)])
def test_norm(kind, d, resid, p):
    torch.manual_seed(d)
    N = 301
    x = torch.randn(N, d, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(N, d, device=DEV, dtype=torch.bfloat16) if resid else None
    w = (1 + 0.1 * torch.randn(d, device=DEV)).to(torch.bfloat16)
    b = (0.1 * torch.randn(d, device=DEV)).to(torch.bfloat16) if kind == norms.LAYER else None
    seed = 1234
    eps = 1e-6
    xs = [t.clone().requires_grad_(True) if t is not None else None for t in (x, r, w, b)]
    out, s = norms._norm(xs[0], xs[1], xs[2], xs[3], eps, p, seed, kind)
    xr = [t.detach().float().clone().requires_grad_(True) if t is not None else None for t in (x, r, w, b)]
    ref_out, ref_s = norms._reference(xr[0], xr[1], xr[2], xr[3], eps, p, seed, kind)
    _close(out, ref_out, 2e-2, 2e-2, "out")
    _close(s, ref_s, 1e-2, 1e-2, "s")
    g1 = torch.randn_like(out)
    g2 = torch.randn_like(out) if (resid or p > 0) else None
    loss = (out.float() * g1.float()).sum() + ((s.float() * g2.float()).sum() if g2 is not None else 0)
    loss.backward()
    ref_loss = (ref_out * g1.float()).sum() + ((ref_s * g2.float()).sum() if g2 is not None else 0)
    ref_loss.backward()
    assert _rel(xs[0].grad, xr[0].grad) < 2e-2
    if resid:
        assert _rel(xs[1].grad, xr[1].grad) < 2e-2
    assert _rel(xs[2].grad, xr[2].grad) < 2e-2
    if b is not None:
        assert _rel(xs[3].grad, xr[3].grad) < 2e-2


@pytest.mark.parametrize("act,gated", [("relu", False), ("gelu", False), ("gelu_new", True), ("gelu_new", False),
                                       ("silu", True)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_act(act, gated, p):
    torch.manual_seed(0)
    N, F = 257, 384
    x = torch.randn(N, 2 * F if gated else F, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = activations.act_dropout(x, act, p, 77, gated=gated)
    xr = x.detach().float().requires_grad_(True)
    yr = activations._reference(xr, act, gated, p, 77)
    _close(y, yr, 2e-2, 2e-2, "act fwd")
    g = torch.randn_like(y)
    (y.float() * g.float()).sum().backward()
    (yr * g.float()).sum().backward()
    assert _rel(x.grad, xr.grad) < 2e-2


def test_dropout_standalone():
    x = torch.randn(64, 96, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    y = activations.dropout(x, 0.25, 99)
    from distributed_llms_example_amd.ops.rng import keep_mask
    ref = x.detach().float() * keep_mask(99, 0.25, x.shape, x.device).float() / 0.75
    _close(y, ref, 1e-2, 1e-2)
    y.sum().backward()
    _close(x.grad, keep_mask(99, 0.25, x.shape, x.device).float() / 0.75, 1e-2, 1e-2)


@pytest.mark.parametrize("V,dtype", [(32128, torch.bfloat16), (50264, torch.bfloat16), (50265, torch.bfloat16),
                                     (1000, torch.bfloat16), (7, torch.bfloat16), (50265, torch.float32),
                                     (1001, torch.float32)])
@pytest.mark.parametrize("smooth,bias", [(0.0, False), (0.1, False), (0.0, True)])
def test_cross_entropy(V, dtype, smooth, bias):
    """Every row alignment: odd V puts row r at an odd element offset (scalar head up to the 16-B boundary, vector
    body, scalar tail); V = 7 is all head."""
    torch.manual_seed(V)
    N = 300
    logits = (3 * torch.randn(N, V, device=DEV)).to(dtype).requires_grad_(True)
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::7] = -100
    bvec = (0.5 * torch.randn(V, device=DEV)) if bias else None
    loss = CE.cross_entropy(logits, labels, bias=bvec, label_smoothing=smooth, inplace_grad=False)
    lr = logits.detach().float().requires_grad_(True)
    ref = CE._reference(lr, labels, bvec, smooth, -100)
    assert abs(loss.item() - ref.item()) < 2e-3 * max(1.0, abs(ref.item()))
    loss.backward()
    ref.backward()
    assert _rel(logits.grad, lr.grad) < 2e-2


def test_cross_entropy_inplace_grad():
    V, N = 32128, 64
    logits = torch.randn(N, V, device=DEV, dtype=torch.bfloat16)
    labels = torch.randint(0, V, (N,), device=DEV)
    lref = logits.float().clone().requires_grad_(True)
    leaf = torch.zeros(N, V, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    x = leaf + logits  # non-leaf produced by an op, like the LM-head GEMM output
    loss = CE.cross_entropy(x, labels, inplace_grad=True)
    loss.backward()
    ref = torch.nn.functional.cross_entropy(lref, labels)
    ref.backward()
    assert _rel(leaf.grad, lref.grad) < 2e-2


def test_adamw_matches_reference():
    from distributed_llms_example_amd.ops.optim import FusedAdamW
    from distributed_llms_example_amd.parallel.flat import FlatParams
    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.LayerNorm(128), torch.nn.Linear(128, 32)).to(DEV)
    m2 = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.LayerNorm(128), torch.nn.Linear(128, 32)).to(DEV)
    m1 = m1.to(torch.bfloat16)
    m2.load_state_dict({k: v.float() for k, v in m1.state_dict().items()})
    f1 = FlatParams(m1)
    opt = FusedAdamW(f1, lr=1e-2, weight_decay=0.01, no_decay=lambda n: "bias" in n or n.startswith("1."))
    ref_groups = [
        {"params": [p for n, p in m2.named_parameters() if not ("bias" in n or n.startswith("1."))], "weight_decay": 0.01},
        {"params": [p for n, p in m2.named_parameters() if ("bias" in n or n.startswith("1."))], "weight_decay": 0.0}]
    ref = torch.optim.AdamW(ref_groups, lr=1e-2)
    for step in range(5):
        x = torch.randn(16, 64, device=DEV)
        loss1 = m1(x.to(torch.bfloat16)).float().pow(2).mean()
        opt.zero_grad()
        loss1.backward()
        # use identical gradients on both sides
        for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
            p2.grad = p1.grad.float().clone()
        norm = opt.step(max_grad_norm=1.0)
        tn = torch.nn.utils.clip_grad_norm_(m2.parameters(), 1.0)
        assert abs(norm.item() - tn.item()) < 1e-2 * tn.item() + 1e-4
        ref.step()
        for p1, p2 in zip(m1.parameters(), m2.parameters()):
            assert _rel(p1, p2) < 1e-2
    # master weights track fp32 reference exactly (up to fp32 rounding)
    for seg, p2 in zip(f1.segments, [p for n, p in reversed(list(m2.named_parameters()))]):
        mw = opt.master[seg.offset:seg.offset + seg.numel].view(seg.shape)
        assert _rel(mw, p2) < 1e-4


ATTN_CASES = [
    # B, H, Sq, Sk, bias, kpm, causal, p, scale
    (2, 4, 128, 128, False, False, False, 0.0, 0.125),
    (2, 3, 200, 200, True, True, False, 0.0, 1.0),
    (1, 2, 77, 300, False, True, False, 0.0, 0.125),   # cross-attention shape
    (2, 2, 130, 130, True, False, True, 0.0, 1.0),     # T5 decoder (causal + unidirectional bias)
    (2, 2, 96, 96, False, False, True, 0.1, 0.125),    # dropout on probabilities
    (1, 2, 257, 257, True, True, False, 0.1, 1.0),
    (1, 2, 1, 33, True, False, True, 0.0, 1.0),        # single-token decode step with cache
    (2, 12, 1024, 1024, True, True, False, 0.1, 1.0),  # t5-base encoder shape
    (2, 3, 300, 600, True, "heavy", False, 0.1, 1.0),  # short dialogue padded to max length: skipped key tiles
    (2, 2, 64, 600, False, "heavy", False, 0.1, 0.125),  # same for cross-attention
    (3, 4, 128, 1000, False, True, False, 0.1, 1.0),   # T5 cross-attention: short-query dK/dV kernel, ragged last block
    (2, 3, 100, 520, False, False, False, 0.1, 0.125),  # same without key padding
]


@pytest.mark.parametrize("B,H,Sq,Sk,bias,kpm,causal,p,scale", ATTN_CASES)
def test_attention(B, H, Sq, Sk, bias, kpm, causal, p, scale, monkeypatch):
    # short-query cross-attention: the dK/dV kernel that walks several key blocks per workgroup, which the launcher
    # otherwise keeps for launches that still fill the chip (csrc/attn.hip attn_bwd_dkdv_sq_kernel)
    monkeypatch.setenv("DLLM_ROUTE", "attn_dkdv_sq_force=1")
    torch.manual_seed(Sq * 7 + Sk)
    D = 64
    q = torch.randn(B, Sq, H, D, device=DEV).to(torch.bfloat16)
    k = torch.randn(B, Sk, H, D, device=DEV).to(torch.bfloat16)
    v = torch.randn(B, Sk, H, D, device=DEV).to(torch.bfloat16)
    table = torch.randn(32, H, device=DEV) * 0.5 if bias else None
    mask = None
    if kpm:
        mask = torch.ones(B, Sk, dtype=torch.bool, device=DEV)
        mask[0, Sk - Sk // 5:] = False
        if kpm == "heavy":  # batch 0: only the first 70 keys are real (whole 64-key tiles / 128-key blocks padded)
            mask[0, 70:] = False
    seed = 4242
    qs, ks, vs = (t.clone().requires_grad_(True) for t in (q, k, v))
    tab1 = table.clone().requires_grad_(True) if bias else None
    lut = A.relative_bias_lut(tab1, Sq, Sk, not causal, 32, 128, q_offset=Sk - Sq) if bias else None
    o = A.attention(qs, ks, vs, scale=scale, causal=causal, key_padding_mask=mask, bias_lut=lut, dropout_p=p, seed=seed)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    tab2 = table.clone().requires_grad_(True) if bias else None
    lut2 = A.relative_bias_lut(tab2, Sq, Sk, not causal, 32, 128, q_offset=Sk - Sq) if bias else None
    ref = A._reference(qr, kr, vr, scale, causal, mask, lut2, p, seed)
    assert _rel(o, ref) < 2e-2, _rel(o, ref)
    g = torch.randn_like(o)
    (o.float() * g.float()).sum().backward()
    (ref * g.float()).sum().backward()
    # a single query row (decode step) makes dq one 64-vector dominated by bf16 rounding of dS
    tol = 6e-2 if Sq < 4 else 3e-2
    for name, a_, b_ in (("dq", qs.grad, qr.grad), ("dk", ks.grad, kr.grad), ("dv", vs.grad, vr.grad)):
        assert _rel(a_, b_) < tol, (name, _rel(a_, b_))
    if bias:
        assert _rel(tab1.grad, tab2.grad) < tol, _rel(tab1.grad, tab2.grad)


def test_attention_packed_qkv_grad():
    B, S, H, D = 2, 150, 4, 64
    qkv = torch.randn(B, S, 3, H, D, device=DEV).to(torch.bfloat16).requires_grad_(True)
    o = A.attention_qkv(qkv, scale=0.125, causal=True)
    r = qkv.detach().float().requires_grad_(True)
    ref = A._reference(r[:, :, 0], r[:, :, 1], r[:, :, 2], 0.125, True, None, None, 0.0, 0)
    assert _rel(o, ref) < 2e-2
    g = torch.randn_like(o)
    (o.float() * g.float()).sum().backward()
    (ref * g.float()).sum().backward()
    assert _rel(qkv.grad, r.grad) < 3e-2
    kvin = torch.randn(B, 70, 2, H, D, device=DEV).to(torch.bfloat16).requires_grad_(True)
    q = torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16).requires_grad_(True)
    o2 = A.attention_q_kv(q, kvin, scale=0.125)
    kr = kvin.detach().float().requires_grad_(True)
    qr = q.detach().float().requires_grad_(True)
    ref2 = A._reference(qr, kr[:, :, 0], kr[:, :, 1], 0.125, False, None, None, 0.0, 0)
    assert _rel(o2, ref2) < 2e-2
    (o2.float().sum()).backward()
    ref2.sum().backward()
    assert _rel(kvin.grad, kr.grad) < 3e-2 and _rel(q.grad, qr.grad) < 3e-2


# ------------------------------------------------------------------------------------ wgrad GEMM
# csrc/gemm_w4.hip weight-gradient mode (variant -1), the only weight-gradient kernel since round 6 (the csrc/gemm.hip
# variants 0-11 were deleted: w4 beat all of them, profiles/r5_wgrad_w4_ab.txt)
@pytest.mark.parametrize("K,M,N,beta,lda_pad", [
    (4096, 768, 768, True, 0),      # t5-base o-proj shape class (many splits)
    (8192, 768, 3072, False, 0),    # wi wgrad, decoder token count
    (2048, 256, 512, True, 64),     # strided A (a column slice of a wider activation)
    (960, 512, 256, True, 0),       # K not a multiple of the split chunk: short last split
    (256, 1024, 2304, False, 0),    # tiles >= CUs / few k-stages: splits == 1, direct bf16 epilogue
])
def test_gemm_wgrad(K, M, N, beta, lda_pad):
    torch.manual_seed(0)
    a_full = torch.randn(K, M + lda_pad, device=DEV, dtype=torch.bfloat16)
    a = a_full[:, lda_pad:] if lda_pad else a_full
    b = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
    c0 = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    c = c0.clone()
    C = _ext.native()
    assert C.gemm_wgrad_supported(a, b, c)
    C.gemm_wgrad(a, b, c, beta, -1, 0)
    ref = a.float().t() @ b.float() + (c0.float() if beta else 0)
    assert _rel(c, ref) < 5e-3, _rel(c, ref)
    _close(c, ref, rtol=2e-2, atol=2e-2 * ref.abs().mean().item(), msg="wgrad")


@pytest.mark.parametrize("K,M,N", [(8192, 768, 2304), (4096, 768, 768), (960, 512, 256)])
def test_gemm_wgrad_deterministic(K, M, N):
    """The split-K weight gradient sums its fp32 slabs in a fixed order (csrc/gemm.hip splitk_reduce_kernel, no
    atomics): 8 repeated runs equal the first bit for bit (a stage buffer read before its DMA landed, or refilled while
    still read, shows up as a mismatch)."""
    torch.manual_seed(K + M)
    a = torch.randn(K, M, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
    C = _ext.native()
    ref = torch.zeros(M, N, device=DEV, dtype=torch.float32)
    C.gemm_wgrad(a, b, ref, False, -1, 0)
    for _ in range(8):
        c = torch.zeros(M, N, device=DEV, dtype=torch.float32)
        C.gemm_wgrad(a, b, c, False, -1, 0)
        assert torch.equal(c, ref)


def test_gemm_wgrad_explicit_splits_match():
    torch.manual_seed(1)
    a = torch.randn(4096, 512, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(4096, 768, device=DEV, dtype=torch.bfloat16)
    outs = []
    for s in (1, 3, 16):
        c = torch.zeros(512, 768, device=DEV, dtype=torch.bfloat16)
        _ext.native().gemm_wgrad(a, b, c, False, -1, s)
        outs.append(c.float())
    ref = a.float().t() @ b.float()
    for o in outs:
        assert _rel(o, ref) < 5e-3


def test_gemm_wgrad_auto_splits_fill_the_last_round():
    """378 output tiles (a t5 LM-head weight gradient: ragged vocab rows x 768) on 256 CUs: one tile per workgroup would
    leave the second round half empty; the auto split count (csrc/bind.cpp wgrad_splits) takes 2 (3 full rounds)."""
    torch.manual_seed(2)
    K, M, N = 8192, 32128, 768
    a = torch.randn(K, M, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
    c = torch.zeros(M, N, device=DEV, dtype=torch.float32)
    splits = _ext.native().gemm_wgrad(a, b, c, False, -1, 0)
    if torch.cuda.get_device_properties(0).multi_processor_count == 256:
        assert splits == 2
    ref = a.float().t() @ b.float()
    assert _rel(c, ref) < 5e-3, _rel(c, ref)


def test_linear_wgrad_path_uses_native_gemm():
    from distributed_llms_example_amd.ops.gemm import _native_ok, wgrad_accumulate
    dy = torch.randn(1024, 768, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(1024, 256, device=DEV, dtype=torch.bfloat16)
    g = torch.zeros(768, 256, device=DEV, dtype=torch.bfloat16)
    assert _native_ok(dy, x, g)
    wgrad_accumulate(g, dy, x)
    wgrad_accumulate(g, dy, x)
    assert _rel(g, 2 * (dy.float().t() @ x.float())) < 5e-3


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("T,N,dt", [(32768, 1024, torch.bfloat16), (1000, 4096, torch.bfloat16), (37, 770, torch.float32),
                                    (4099, 3072, torch.float32)])
def test_colsum_acc_bias_grad(T, N, dt, aligned):
    """aligned: 16-B rows (8 columns per lane); else strided rows at a 4-B offset (2 columns per lane)."""
    torch.manual_seed(0)
    x_full = torch.randn(T, N + 8, device=DEV, dtype=torch.bfloat16)
    x = x_full[:, :N] if aligned else x_full[:, 2:N + 2]
    out0 = torch.randn(N, device=DEV, dtype=dt)
    out = out0.clone()
    _ext.native().colsum_acc(x, out)
    ref = out0.float() + x.float().sum(0)
    _close(out, ref, rtol=1e-2, atol=1e-2 * (T ** 0.5) / 10 + 1e-2, msg="colsum")


def test_attention_prefetched_dropout_planes_match(monkeypatch):
    """Keep bits generated ahead on the side stream == bits hashed inside the forward (same seed)."""
    B, S, H, D, p, seed = 2, 200, 3, 64, 0.1, 99
    torch.manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, device=DEV).to(torch.bfloat16)
    g = torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16)
    outs = []
    for use_pre in (False, True):
        x = qkv.clone().requires_grad_(True)
        pre = A.prefetch_dropout_mask(x, B, H, S, S, p, seed) if use_pre else None
        assert (pre is not None) == use_pre
        o = A.attention_qkv(x, pre=pre, scale=0.125, dropout_p=p, seed=seed)
        o.backward(g)
        outs.append((o.detach(), x.grad))
    torch.testing.assert_close(outs[0][0], outs[1][0], rtol=0, atol=0)
    torch.testing.assert_close(outs[0][1], outs[1][1], rtol=0, atol=0)


# ------------------------------------------------------------------------ fused-epilogue GEMM (csrc/gemm_fused.hip)
_EPI_FWD = {None: 0, "relu": 1, "gelu": 2, "gelu_new": 5}
_EPI_BWD = {"relu": 3, "gelu": 4, "gelu_new": 6}


@pytest.mark.parametrize("variant", [1, 8, 9])  # 1: 128x128 single-wave-group, 8: ping-pong, 9: persistent ping-pong
@pytest.mark.parametrize("act,p,bias", [(None, 0.0, False), ("relu", 0.1, False), ("gelu", 0.0, True),
                                        ("gelu_new", 0.1, True)])
def test_gemm_fused_forward(variant, act, p, bias):
    """H = dropout(act(X Wᵀ + b)) with the epilogue in the GEMM (nn.Linear weight layout) vs fp32 torch."""
    torch.manual_seed(0)
    M, K, N = 512, 768, 1280
    C = _ext.native()
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    b = (0.5 * torch.randn(N, device=DEV)).to(torch.bfloat16) if bias else None
    epi = _EPI_FWD[act]
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16) if epi in (2, 5) else None
    assert C.gemm_fused_supported(x, w, False)
    h = C.gemm_fused(x, w, False, epi, b, None, aux, p, 77, variant)
    u = x.float() @ w.float().t() + (b.float() if bias else 0.0)
    ref = u if act is None else activations._act_ref(u, act)
    if p > 0:
        ref = ref * activations.ffn_keep_mask(act, False, 77, p, ref.shape, ref.device).float() / (1.0 - p)
    assert _rel(h, ref) < 1e-2, _rel(h, ref)
    _close(h, ref, 2e-2, 2e-2, "fused fwd")
    if aux is not None:  # GELU: the derivative with the dropout mask and scale applied (the backward's multiplier)
        assert _rel(aux, _act_grad(u, act, 77, p)) < 1e-2, _rel(aux, _act_grad(u, act, 77, p))


def _act_grad(u, act, seed, p):
    """act'(u) * dropout'(.) in fp32 (what the GELU forward epilogues write as their second output)."""
    uf = u.float().requires_grad_(True)
    activations._act_ref(uf, act).sum().backward()
    g = uf.grad
    if p > 0:
        g = g * activations.ffn_keep_mask(act, False, seed, p, g.shape, g.device).float() / (1.0 - p)
    return g


@pytest.mark.parametrize("variant", [1, 8, 9])
@pytest.mark.parametrize("act,p", [("relu", 0.1), ("relu", 0.0), ("gelu", 0.1), ("gelu_new", 0.0)])
def test_gemm_fused_backward(variant, act, p):
    """dU = act'(U) * dropout'(dY Wo) with Wo k-major ([d, F]) vs fp32 autograd of the same composite."""
    torch.manual_seed(1)
    M, d, F_ = 768, 512, 1024
    C = _ext.native()
    dy = torch.randn(M, d, device=DEV).to(torch.bfloat16)
    wo = (torch.randn(d, F_, device=DEV) * d ** -0.5).to(torch.bfloat16)
    u = torch.randn(M, F_, device=DEV).to(torch.bfloat16)
    keep = (activations.ffn_keep_mask(act, False, 9, p, (M, F_), u.device).float() / (1.0 - p)) if p > 0 else \
        torch.ones(M, F_, device=DEV)
    h = (activations._act_ref(u.float(), act) * keep).to(torch.bfloat16)
    # ReLU derives its mask from the saved activation itself; GELU multiplies by the derivative its forward stored
    aux = h if act == "relu" else _act_grad(u, act, 9, p).to(torch.bfloat16)
    assert C.gemm_fused_supported(dy, wo, True)
    du = C.gemm_fused(dy, wo, True, _EPI_BWD[act], None, aux, None, p, 9, variant)
    uf = u.float().requires_grad_(True)
    (activations._act_ref(uf, act) * keep).backward(dy.float() @ wo.float())
    assert _rel(du, uf.grad) < 1e-2, _rel(du, uf.grad)
    _close(du, uf.grad, 2e-2, 2e-2, "fused bwd")


@pytest.mark.parametrize("variant", [1, 8, 9])
@pytest.mark.parametrize("K", [64, 128, 192, 320])
def test_gemm_fused_short_k(variant, K):
    """Pipeline prologue / tail paths: k-tile counts 1..5 (fewer k-tiles than the DMA ring holds)."""
    torch.manual_seed(2)
    M, N = 768, 512
    C = _ext.native()
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    h = C.gemm_fused(x, w, False, 0, None, None, None, 0.0, 1, variant)
    _close(h, x.float() @ w.float().t(), 2e-2, 2e-2, "short-k")


@pytest.mark.parametrize("grp", [1, 2, 3, 4, 8])
def test_gemm_pp_tile_order_groups(grp, monkeypatch):
    """Grouped tile order of the ping-pong kernel (routing gemm_grp), including a last group shorter than grp."""
    monkeypatch.setenv("DLLM_ROUTE", f"gemm_grp={grp}")
    torch.manual_seed(3)
    M, K, N = 1280, 256, 768
    C = _ext.native()
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    h = C.gemm_fused(x, w, False, 1, None, None, None, 0.0, 1, 8)
    _close(h, torch.relu(x.float() @ w.float().t()), 2e-2, 2e-2, "pp grouped order")


@pytest.mark.parametrize("K", [128, 192, 768])
@pytest.mark.parametrize("kmajor", [False, True])
def test_gemm_pp_persistent(K, kmajor):
    """Persistent ping-pong kernel (variant 9: one workgroup per CU walking >= 2 tiles, the DMA stream running across
    tile boundaries, epilogue stores queued between units): 528 tiles (uneven per CU), relu+dropout forward (NT) or
    d-relu backward (k-major B), vs the fp32 reference."""
    from distributed_llms_example_amd.ops.rng import keep_mask
    torch.manual_seed(4)
    M, N, p = 8448, 4096, 0.1
    C = _ext.native()
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    if not kmajor:
        w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
        h = C.gemm_fused(x, w, False, 1, None, None, None, p, 5, 9)
        ref = torch.relu(x.float() @ w.float().t()) * activations.ffn_keep_mask("relu", False, 5, p, (M, N),
                                                                                x.device).float() / (1.0 - p)
        _close(h, ref, 2e-2, 2e-2, "pp persistent fwd")
    else:
        w = (torch.randn(K, N, device=DEV) * K ** -0.5).to(torch.bfloat16)
        hs = (torch.relu(torch.randn(M, N, device=DEV)) * keep_mask(6, p, (M, N), x.device).float()).to(torch.bfloat16)
        du = C.gemm_fused(x, w, True, 3, None, hs, None, p, 6, 9)
        ref = (x.float() @ w.float()) * (hs.float() != 0).float() / (1.0 - p)
        _close(du, ref, 2e-2, 2e-2, "pp persistent bwd")


@pytest.mark.parametrize("act,p", [("gelu", 0.1), ("gelu", 0.0), ("gelu_new", 0.1)])
def test_gemm_pp_persistent_gelu(act, p):
    """GELU forward (bias + dropout, two stores: H and the scaled derivative) on the persistent ping-pong kernel: 528
    tiles over the CUs, so every workgroup runs an epilogue inside the DMA stream of its next tile."""
    torch.manual_seed(6)
    M, K, N = 8448, 1024, 4096
    C = _ext.native()
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    b = (0.5 * torch.randn(N, device=DEV)).to(torch.bfloat16)
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    h = C.gemm_fused(x, w, False, _EPI_FWD[act], b, None, aux, p, 31, 9)
    u = x.float() @ w.float().t() + b.float()
    ref = activations._act_ref(u, act)
    if p > 0:
        ref = ref * activations.ffn_keep_mask(act, False, 31, p, ref.shape, ref.device).float() / (1.0 - p)
    _close(h, ref, 2e-2, 2e-2, "pp persistent gelu fwd")
    assert _rel(aux, _act_grad(u, act, 31, p)) < 1e-2, _rel(aux, _act_grad(u, act, 31, p))


@pytest.mark.parametrize("variant", [8, 9])
@pytest.mark.parametrize("M,d,F_", [(768, 512, 1024), (8448, 768, 4096)])
def test_gemm_relu_bit_mask(variant, M, d, F_):
    """ReLU derivative bits: the forward (epi 1) writes them next to H, the backward (epi 7) stages them through LDS;
    both outputs must equal the aux-tensor path (epi 1 without mask / epi 3 reading H) bit for bit."""
    torch.manual_seed(5)
    p = 0.1
    C = _ext.native()
    x = torch.randn(M, d, device=DEV).to(torch.bfloat16)
    wi = (torch.randn(F_, d, device=DEV) * d ** -0.5).to(torch.bfloat16)
    bi = (0.1 * torch.randn(F_, device=DEV)).to(torch.bfloat16)
    mask = torch.full((M * F_ // 32,), -1, device=DEV, dtype=torch.int32)
    h0 = C.gemm_fused(x, wi, False, 1, bi, None, None, p, 11, variant)
    h = C.gemm_fused(x, wi, False, 1, bi, None, None, p, 11, variant, mask)
    torch.testing.assert_close(h, h0, rtol=0, atol=0)
    dy = torch.randn(M, d, device=DEV).to(torch.bfloat16)
    wo = (torch.randn(d, F_, device=DEV) * d ** -0.5).to(torch.bfloat16)
    du0 = C.gemm_fused(dy, wo, True, 3, None, h, None, p, 11, variant)
    du = C.gemm_fused(dy, wo, True, 7, None, None, None, p, 11, variant, mask)
    torch.testing.assert_close(du, du0, rtol=0, atol=0)
    assert (du == 0).float().mean().item() > 0.4  # the mask really zeroes (ReLU ~ half, dropout 10 %)
    with pytest.raises(RuntimeError):
        C.gemm_fused(dy, wo, True, 7, None, None, None, p, 11, 1, mask)  # mask needs the ping-pong kernel


def _geglu_ref(gate, up, seed, p):
    """fp32 h = dropout(gelu_tanh(gate) * up) and the two factors the gated forward epilogue stores."""
    s = (activations.ffn_keep_mask("gelu_new", True, seed, p, gate.shape, gate.device).float() / (1.0 - p)) if p > 0 \
        else torch.ones_like(gate)
    g = gate.detach().float().clone().requires_grad_(True)
    a = activations._act_ref(g, "gelu_new")
    (da,) = torch.autograd.grad(a.sum(), g)
    a = a.detach()
    return a * up * s, da * up * s, a * s


@pytest.mark.parametrize("M,d,F_", [(512, 768, 1024), (768, 512, 1280), (2048, 2048, 5120), (4096, 1024, 4096)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm_geglu_forward(M, d, F_, p):
    """Gated-GELU input GEMM (epi 8): one GEMM over the stacked [wi_0; wi_1] whose epilogue pairs gate and up columns
    in registers (4096 x 4096: 512 tiles, the persistent launch); h, G1 = s·gelu'(gate)·up, G2 = s·gelu(gate) vs fp32 torch (same counter-hash dropout mask as
    csrc/act.hip's gated path)."""
    torch.manual_seed(6)
    C = _ext.native()
    x = torch.randn(M, d, device=DEV).to(torch.bfloat16)
    wi = (torch.randn(2 * F_, d, device=DEV) * d ** -0.5).to(torch.bfloat16)
    h, g1, g2 = C.gemm_geglu(x, wi, p, 21)
    u = x.float() @ wi.float().t()
    rh, r1, r2 = _geglu_ref(u[:, :F_], u[:, F_:], 21, p)
    for name, got, ref in (("h", h, rh), ("G1", g1, r1), ("G2", g2, r2)):
        assert _rel(got, ref) < 1e-2, (name, _rel(got, ref))
        _close(got, ref, 2e-2, 2e-2, f"geglu {name}")
    if p > 0:  # the unfused path (hipBLASLt + csrc/act.hip gated kernel) drops exactly the same elements
        dropped = ~activations.ffn_keep_mask("gelu_new", True, 21, p, (M, F_), x.device)
        h_unf = activations.act_dropout(x @ wi.t(), "gelu_new", p, 21, gated=True)
        assert bool((h[dropped] == 0).all()) and bool((h_unf[dropped] == 0).all())
        assert _rel(h_unf, h) < 1e-2


@pytest.mark.parametrize("M,d,F_", [(512, 768, 1024), (768, 512, 1280), (8192, 1024, 4096)])
def test_gemm_geglu_backward(M, d, F_):
    """Gated backward GEMM (epi 9): dH = dy · wo (k-major wo [d, F]) -> [dH·G1 | dH·G2] in the stacked [M, 2F] layout,
    vs fp32 autograd of the gated composite."""
    torch.manual_seed(7)
    p = 0.1
    C = _ext.native()
    gate = torch.randn(M, F_, device=DEV)
    up = torch.randn(M, F_, device=DEV)
    _, r1, r2 = _geglu_ref(gate, up, 33, p)
    g1, g2 = r1.to(torch.bfloat16), r2.to(torch.bfloat16)
    dy = torch.randn(M, d, device=DEV).to(torch.bfloat16)
    wo = (torch.randn(d, F_, device=DEV) * d ** -0.5).to(torch.bfloat16)
    du = C.gemm_dgeglu(dy, wo, g1, g2)
    dh = dy.float() @ wo.float()
    ref = torch.cat([dh * g1.float(), dh * g2.float()], dim=1)
    assert du.shape == (M, 2 * F_)
    assert _rel(du, ref) < 1e-2, _rel(du, ref)
    _close(du, ref, 2e-2, 2e-2, "dgeglu")
    # end to end against autograd of dropout(gelu(gate) * up)
    gf, uf = gate.detach().clone().requires_grad_(True), up.detach().clone().requires_grad_(True)
    keep = activations.ffn_keep_mask("gelu_new", True, 33, p, (M, F_), gate.device).float() / (1.0 - p)
    (activations._act_ref(gf, "gelu_new") * uf * keep).backward(dh)
    assert _rel(du, torch.cat([gf.grad, uf.grad], dim=1)) < 2e-2


@pytest.mark.parametrize("variant", [8, 9])
@pytest.mark.parametrize("act,M,d,F_", [("gelu", 768, 512, 1024), ("gelu_new", 8448, 1024, 4096)])
def test_gemm_fused_gelu_bwd_colsum(variant, act, M, d, F_):
    """GELU backward GEMM epilogue also writes per-128-row column sums of dU (the fc1 bias gradient) vs fp32 sums."""
    torch.manual_seed(9)
    C = _ext.native()
    dy = torch.randn(M, d, device=DEV).to(torch.bfloat16)
    wo = (torch.randn(d, F_, device=DEV) * d ** -0.5).to(torch.bfloat16)
    u = torch.randn(M, F_, device=DEV).to(torch.bfloat16)
    aux = _act_grad(u, act, 9, 0.1).to(torch.bfloat16)
    part = torch.full((M // 128, F_), float("nan"), device=DEV)
    du = C.gemm_fused(dy, wo, True, _EPI_BWD[act], None, aux, None, 0.1, 9, variant, None, part)
    du0 = C.gemm_fused(dy, wo, True, _EPI_BWD[act], None, aux, None, 0.1, 9, variant)
    torch.testing.assert_close(du, du0, rtol=0, atol=0)
    ref = du.float().view(M // 128, 128, F_).sum(1)  # sums of the stored (bf16-rounded) values: fp32 accumulators
    assert _rel(part, ref) < 1e-2, _rel(part, ref)
    assert _rel(part.sum(0), du.float().sum(0)) < 1e-2


def test_gemm_fused_rejects_unsupported_shapes():
    C = _ext.native()
    x = torch.randn(300, 768, device=DEV).to(torch.bfloat16)  # tokens not a multiple of 256
    w = torch.randn(1024, 768, device=DEV).to(torch.bfloat16)
    assert not C.gemm_fused_supported(x, w, False)
    with pytest.raises(RuntimeError):
        C.gemm_fused(x, w, False, 1, None, None, None, 0.0, 0, -1)


@pytest.mark.parametrize("causal,S", [(False, 1024), (True, 384), (False, 300)])
def test_attention_saturated_bias_tiles_match(causal, S):
    """relative_bias_lut's LUT declares its constant-bucket ranges; the kernels' scalar-bias tiles and end-of-range
    dS credit must give the same outputs and the same per-bucket table gradient as the full LUT path."""
    torch.manual_seed(0)
    B, H, D, p = 2, 4, 64, 0.1
    qkv = torch.randn(B, S, 3, H, D, device=DEV).to(torch.bfloat16)
    g = torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16)
    table = torch.randn(32, H, device=DEV)
    outs = []
    for use_sat in (False, True):
        tb = table.clone().requires_grad_(True)
        lut = A.relative_bias_lut(tb, S, S, not causal, 32, 128)
        assert lut._dllm_sat[0] >= 0
        if not use_sat:
            lut._dllm_sat = None
        x = qkv.clone().requires_grad_(True)
        o = A.attention_qkv(x, bias_lut=lut, causal=causal, scale=1.0, dropout_p=p, seed=3)
        o.backward(g)
        outs.append((o.detach().float(), x.grad.float(), tb.grad.clone()))
    (o0, gx0, gt0), (o1, gx1, gt1) = outs
    assert _rel(o1, o0) < 1e-3, _rel(o1, o0)
    assert _rel(gx1, gx0) < 1e-3, _rel(gx1, gx0)
    assert _rel(gt1, gt0) < 1e-3, _rel(gt1, gt0)


@pytest.mark.parametrize("W,S,p", [(2, 512, 0.0), (4, 256, 0.0), (2, 384, 0.1)])
def test_context_parallel_blocks(W, S, p):
    """Ring attention numerics on one GPU: W virtual ranks run the native flash kernels per (q shard, kv shard)
    block with global-distance T5 bias LUTs, merge by LSE, and run the backward per block with the global
    o / lse (parallel/context.py); p = 0 must equal the unsharded fp32 attention, p > 0 its per-block-seed
    reference."""
    from distributed_llms_example_amd.parallel import context as cp
    torch.manual_seed(W * 1000 + S)
    B, H, D = 2, 4, 64
    N = W * S
    q, k, v = (torch.randn(B, N, H, D, device=DEV).to(torch.bfloat16) for _ in range(3))
    table = torch.randn(32, H, device=DEV) * 0.5
    mask = torch.ones(B, N, dtype=torch.bool, device=DEV)
    mask[1, N - S // 2 - 7:] = False
    km = mask.to(torch.uint8)
    do = torch.randn(B, N, H, D, device=DEV).to(torch.bfloat16)
    seed = 99
    outs, lses = [], []
    luts = {}
    for r in range(W):
        qr = q[:, r * S:(r + 1) * S]
        o_acc = l_acc = None
        for s in range(W):
            lt = A.relative_bias_lut(table, S, S, True, 32, 128, q_offset=(r - s) * S)
            luts[(r, s)] = lt
            o_b, l_b, _ = cp._block_fwd(qr, k[:, s * S:(s + 1) * S], v[:, s * S:(s + 1) * S],
                                        km[:, s * S:(s + 1) * S].contiguous(), lt, lt._dllm_sat, 1.0, p,
                                        cp._block_seed(seed, r, s))
            o_acc, l_acc = (o_b, l_b) if o_acc is None else cp._merge(o_acc, l_acc, o_b, l_b)
        outs.append(o_acc.to(torch.bfloat16))
        lses.append(l_acc.contiguous())
    o = torch.cat(outs, 1)
    dq = torch.zeros(B, N, H, D, device=DEV)
    dk = torch.zeros_like(dq)
    dv = torch.zeros_like(dq)
    dlut = {}
    for r in range(W):
        for s in range(W):
            lt = luts[(r, s)]
            sl_q, sl_k = slice(r * S, (r + 1) * S), slice(s * S, (s + 1) * S)
            dmask = None
            if p > 0:  # the planes the forward would have produced for this block
                dmask = _ext.native().attn_dropout_mask(B, H, S, S, p, cp._block_seed(seed, r, s), q)
            a, b_, c, dl = cp._block_bwd(do[:, sl_q].contiguous(), q[:, sl_q], k[:, sl_k], v[:, sl_k],
                                         outs[r], lses[r], km[:, sl_k].contiguous(), lt, lt._dllm_sat, 1.0, p,
                                         cp._block_seed(seed, r, s), True, dmask)
            dq[:, sl_q] += a
            dk[:, sl_k] += b_
            dv[:, sl_k] += c
            dlut[(r, s)] = dl
    # fp32 reference of the same math
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    tab = table.clone().requires_grad_(True)
    if p == 0.0:
        ref = A._reference(qf, kf, vf, 1.0, False, mask, A.relative_bias_lut(tab, N, N, True, 32, 128), 0.0, 0)
    else:
        rows = []
        for r in range(W):
            o_acc = l_acc = None
            for s in range(W):
                lt = A.relative_bias_lut(tab, S, S, True, 32, 128, q_offset=(r - s) * S)
                o_b, l_b = cp._ref_block_fwd(qf[:, r * S:(r + 1) * S], kf[:, s * S:(s + 1) * S],
                                             vf[:, s * S:(s + 1) * S], mask[:, s * S:(s + 1) * S], lt, 1.0, p,
                                             cp._block_seed(seed, r, s))
                o_acc, l_acc = (o_b, l_b) if o_acc is None else cp._merge(o_acc, l_acc, o_b, l_b)
            rows.append(o_acc)
        ref = torch.cat(rows, 1)
    assert _rel(o, ref) < 2e-2, _rel(o, ref)
    ref.backward(do.float())
    for name, a_, b_ in (("dq", dq, qf.grad), ("dk", dk, kf.grad), ("dv", dv, vf.grad)):
        assert _rel(a_, b_) < 3e-2, (name, _rel(a_, b_))
    # bucket-table gradient through the W x W global-distance LUTs
    tg = table.clone().requires_grad_(True)
    tot = sum((A.relative_bias_lut(tg, S, S, True, 32, 128, q_offset=(r - s) * S) * dlut[(r, s)]).sum()
              for r in range(W) for s in range(W))
    tot.backward()
    assert _rel(tg.grad, tab.grad) < 3e-2, _rel(tg.grad, tab.grad)


def test_ring_attention_single_rank_equals_attention():
    """ring_attention with no process group (W = 1) runs one native block: same as attention() incl. grads."""
    from distributed_llms_example_amd.parallel.context import ring_attention
    torch.manual_seed(3)
    B, S, H, D = 2, 320, 4, 64
    q, k, v = (torch.randn(B, S, H, D, device=DEV).to(torch.bfloat16) for _ in range(3))
    mask = torch.ones(B, S, dtype=torch.bool, device=DEV)
    mask[0, 250:] = False
    table = torch.randn(32, H, device=DEV) * 0.5
    t1, t2 = table.clone().requires_grad_(True), table.clone().requires_grad_(True)
    a = [t.clone().requires_grad_(True) for t in (q, k, v)]
    b = [t.clone().requires_grad_(True) for t in (q, k, v)]
    o1 = ring_attention(*a, key_padding_mask=mask, bias_table=t1)
    o2 = A.attention(*b, key_padding_mask=mask, bias_lut=A.relative_bias_lut(t2, S, S, True, 32, 128))
    assert _rel(o1, o2) < 1e-2
    g = torch.randn_like(o1)
    (o1.float() * g.float()).sum().backward()
    (o2.float() * g.float()).sum().backward()
    for x, y in zip(a + [t1], b + [t2]):
        assert _rel(x.grad, y.grad) < 2e-2, _rel(x.grad, y.grad)


def test_chunked_attention_long_sequence():
    """Single-GPU long encoder: 4K-token blocks merged by LSE equal the single kernel at 8K and the fp32
    reference at 16K (beyond the single kernel's LDS-bounded length)."""
    from distributed_llms_example_amd.parallel.context import chunked_attention
    torch.manual_seed(11)
    for N, H, full in ((8192, 4, "kernel"), (16384, 2, "reference")):
        B, D = 1, 64
        q, k, v = (torch.randn(B, N, H, D, device=DEV).to(torch.bfloat16) for _ in range(3))
        mask = torch.ones(B, N, dtype=torch.bool, device=DEV)
        mask[0, N - 1000:] = False
        table = torch.randn(32, H, device=DEV) * 0.5
        t1, t2 = table.clone().requires_grad_(True), table.clone().requires_grad_(True)
        a = [t.clone().requires_grad_(True) for t in (q, k, v)]
        o1 = chunked_attention(*a, chunk=4096, key_padding_mask=mask, bias_table=t1)
        if full == "kernel":
            b = [t.clone().requires_grad_(True) for t in (q, k, v)]
            o2 = A.attention(*b, key_padding_mask=mask, bias_lut=A.relative_bias_lut(t2, N, N, True, 32, 128))
        else:
            b = [t.float().requires_grad_(True) for t in (q, k, v)]
            o2 = A._reference(*b, 1.0, False, mask, A.relative_bias_lut(t2, N, N, True, 32, 128), 0.0, 0)
        assert _rel(o1, o2) < 2e-2, (N, _rel(o1, o2))
        g = torch.randn_like(o1)
        (o1.float() * g.float()).sum().backward()
        (o2.float() * g.float()).sum().backward()
        # vs the fp32 reference the bf16 dS rounding over 16K keys costs a little more than at 1K (3e-2)
        tol = 3e-2 if full == "kernel" else 5e-2
        for name, x, y in zip(("dq", "dk", "dv", "dtable"), a + [t1], b + [t2]):
            assert _rel(x.grad, y.grad) < tol, (N, name, _rel(x.grad, y.grad))
        del o2, b
        torch.cuda.empty_cache()


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_chunked_attention_8k_blocks_vs_fp32(p):
    """The default long-sequence path at batch x heads < 32 (8K-token blocks, parallel/context.py
    long_sequence_chunk) vs an fp32 reference of the same block math at 16K tokens: off-diagonal bias LUTs with
    saturated ranges, key padding, attention dropout (per-block seeds); outputs and dq / dk / dv / dtable."""
    from distributed_llms_example_amd.parallel import context as cp
    torch.manual_seed(12)
    B, N, H, D = 1, 16384, 2, 64
    chunk = cp.long_sequence_chunk(N, rows=B * H)
    assert chunk == 8192, chunk
    q, k, v = (torch.randn(B, N, H, D, device=DEV).to(torch.bfloat16) for _ in range(3))
    mask = torch.ones(B, N, dtype=torch.bool, device=DEV)
    mask[0, N - 1500:] = False
    table = torch.randn(32, H, device=DEV) * 0.5
    seed = 4321
    t1 = table.clone().requires_grad_(True)
    a = [t.clone().requires_grad_(True) for t in (q, k, v)]
    o = cp.chunked_attention(*a, chunk=chunk, key_padding_mask=mask, bias_table=t1, dropout_p=p, seed=seed)
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    tab = table.clone().requires_grad_(True)
    W, S = N // chunk, chunk
    rows = []
    for r in range(W):
        o_acc = l_acc = None
        for s in range(W):
            lt = A.relative_bias_lut(tab, S, S, True, 32, 128, q_offset=(r - s) * S)
            o_b, l_b = cp._ref_block_fwd(qf[:, r * S:(r + 1) * S], kf[:, s * S:(s + 1) * S], vf[:, s * S:(s + 1) * S],
                                         mask[:, s * S:(s + 1) * S], lt, 1.0, p, cp._block_seed(seed, r, s))
            o_acc, l_acc = (o_b, l_b) if o_acc is None else cp._merge(o_acc, l_acc, o_b, l_b)
        rows.append(o_acc)
    ref = torch.cat(rows, 1)
    assert _rel(o, ref) < 2e-2, _rel(o, ref)
    g = torch.randn_like(ref)
    (o.float() * g).sum().backward()
    (ref * g).sum().backward()
    for name, x, y in zip(("dq", "dk", "dv", "dtable"), a + [t1], [qf, kf, vf, tab]):
        assert _rel(x.grad, y.grad) < 5e-2, (name, _rel(x.grad, y.grad))


@pytest.mark.parametrize("rows,native", [(1024, False), (4096, True)])
def test_wgrad_small_rows_route(rows, native, monkeypatch):
    """routing wgrad_min_rows (default 4096): below it the weight gradient is the library's fp32 addmm into the fp32
    gradient (accumulated, beta); from it the w4 weight-gradient mode.  Both equal the fp64 product."""
    from distributed_llms_example_amd.ops import gemm as gemm_mod
    monkeypatch.setenv("DLLM_ROUTE", "wgrad_min_rows=4096")
    torch.manual_seed(7)
    dy = torch.randn(rows, 768, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(rows, 512, device=DEV, dtype=torch.bfloat16)
    g0 = torch.randn(768, 512, device=DEV, dtype=torch.float32)
    g = g0.clone()
    calls = []
    monkeypatch.setattr(gemm_mod, "_native_ok", lambda *a: calls.append(1) or True)
    gemm_mod._wgrad(g, dy, x, True)
    assert (len(calls) > 0) == native
    ref = g0.double() + dy.double().t() @ x.double()
    assert _rel(g, ref) < 1e-5, _rel(g, ref)


@pytest.mark.parametrize("G,d", [(512, 768), (2048, 1024), (8192, 768), (4100, 520)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_colsum_partials_acc(G, d, out_dtype):
    """out += part.sum(0) over fp32 partial rows (norm-weight / bias gradients; a deferred accumulation window hands
    thousands of rows), fp32 or bf16 destination, deterministic, vs fp64."""
    torch.manual_seed(G + d)
    C = _ext.native()
    part = torch.randn(G, d, device=DEV)
    base = torch.randn(d, device=DEV).to(out_dtype)
    out = base.clone()
    C.colsum_partials_acc(part, out)
    ref = base.double() + part.double().sum(0)
    if out_dtype == torch.float32:  # fp32 summation error, bounded against the column's L1 mass
        assert ((out.double() - ref).abs() / part.double().abs().sum(0)).max().item() < 2e-6
    else:  # the bf16 store's rounding
        assert ((out.double() - ref).abs() / ref.abs().clamp_min(1.0)).max().item() < 1e-2
    out2 = base.clone()
    C.colsum_partials_acc(part, out2)
    assert torch.equal(out, out2)  # run-to-run identical
