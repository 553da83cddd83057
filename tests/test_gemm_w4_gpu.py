"""One-wave-per-SIMD projection GEMM (csrc/gemm_w4.hip) vs a plain-PyTorch fp32 reference of the same op.

Covers NT (forward: b = nn.Linear weight [N, K]) and NN (input gradient: b = [K, N] k-major), bias, accumulate
(out += a . b), ragged M / N (loads past the edge read 0 through the buffer descriptor, stores masked), strided
operands and an output view inside a larger buffer (nothing outside the view may be written).
"""
import pytest
import torch

from distributed_llms_example_amd import _ext

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


SHAPES = [(256, 64, 256), (512, 128, 512), (300, 192, 264), (1000, 768, 2304), (64, 64, 8), (257, 64, 520),
          (4096, 1024, 1024), (768, 3072, 768),
          # > 256 tiles: the persistent form (one workgroup per CU walking 1-2 tiles, DMA crossing tile boundaries;
          # K = 128 crosses at every other k-tile), ragged M / N on the last tiles
          (8192, 128, 2304), (9000, 192, 2000), (70000, 64, 264)]


@pytest.mark.parametrize("M,K,N", SHAPES)
@pytest.mark.parametrize("kmajor", [False, True])
@pytest.mark.parametrize("bias,acc", [(False, False), (True, False), (False, True), (True, True)])
def test_gemm_w4(M, K, N, kmajor, bias, acc):
    C = _ext.native()
    torch.manual_seed(M * 7 + K * 3 + N)
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    b = w.t().contiguous() if kmajor else w
    bv = torch.randn(N, device=DEV).to(torch.bfloat16) if bias else None
    out = torch.randn(M, N, device=DEV).to(torch.bfloat16) if acc else None
    ref = a.float() @ w.float().t()
    if bias:
        ref = ref + bv.float()
    if acc:
        ref = ref + out.float()
    assert C.gemm_w4_supported(a, b, kmajor)
    got = C.gemm_w4(a, b, kmajor, bv, out, acc)
    if not acc:  # one tile per workgroup: the same numbers
        again = C.gemm_w4(a, b, kmajor, bv, None, False, -1, False)
        assert torch.equal(again, got)
    if acc:
        assert got.data_ptr() == out.data_ptr()
    assert got.shape == (M, N)
    assert torch.isfinite(got.float()).all()
    assert _rel(got, ref) < 8e-3, _rel(got, ref)


@pytest.mark.parametrize("kmajor", [False, True])
def test_gemm_w4_strided_views(kmajor):
    """lda / ldb / ldc larger than the logical rows, output a view: the guard band around it stays untouched."""
    C = _ext.native()
    M, K, N = 520, 256, 392
    a_full = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)
    a = a_full[:, 32:32 + K]
    if kmajor:
        b_full = torch.randn(K, N + 24, device=DEV).to(torch.bfloat16) * K ** -0.5
        b = b_full[:, 8:8 + N]
        wref = b.float().t()
    else:
        b_full = torch.randn(N, K + 128, device=DEV).to(torch.bfloat16) * K ** -0.5
        b = b_full[:, 64:64 + K]
        wref = b.float()
    guard = torch.full((M + 3, N + 40), 7.0, device=DEV, dtype=torch.bfloat16)
    out = guard[1:1 + M, 16:16 + N]
    C.gemm_w4(a, b, kmajor, None, out, False)
    ref = a.float() @ wref.t()
    assert _rel(out, ref) < 8e-3
    mask = torch.ones_like(guard, dtype=torch.bool)
    mask[1:1 + M, 16:16 + N] = False
    assert (guard[mask] == 7.0).all(), "gemm_w4 wrote outside its output view"


def test_gemm_w4_rejects_bad_shapes():
    C = _ext.native()
    a = torch.randn(256, 100, device=DEV).to(torch.bfloat16)  # K % 64 != 0
    w = torch.randn(256, 100, device=DEV).to(torch.bfloat16)
    assert not C.gemm_w4_supported(a, w, False)
    with pytest.raises(RuntimeError):
        C.gemm_w4(a, w, False)


@pytest.mark.parametrize("M,K,N", [(512, 128, 512), (1000, 768, 3072), (9000, 192, 2000), (300, 64, 264)])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_w4_relu_dropout_mask_roundtrip(M, K, N, p, bias):
    """T5 FFN on w4 (ops/ffn.py): forward H = dropout(relu(X Wiᵀ + b)) with the row-Weyl keep decision of (row m,
    column n) (ops/rng.py rowwise_keep_mask), writing the keep-and-positive bit mask; backward dU = (dY Wo) * mask /
    (1-p) read from that mask.  Both vs fp32 torch."""
    from distributed_llms_example_amd.ops.rng import rowwise_keep_mask
    C = _ext.native()
    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    wi = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    bi = torch.randn(N, device=DEV).to(torch.bfloat16) if bias else None
    seed = 1234
    mask = torch.zeros(C.gemm_w4_mask_words(M, N), device=DEV, dtype=torch.int32)
    h = C.gemm_w4(x, wi, False, bi, None, False, -1, True, 1, p, seed, mask)
    u = x.float() @ wi.float().t() + (bi.float() if bias else 0.0)
    keep = rowwise_keep_mask(seed, p, M, N, DEV) if p > 0 else torch.ones(M, N, dtype=torch.bool, device=DEV)
    ref = torch.relu(u) * keep / (1 - p)
    assert _rel(h, ref) < 8e-3, _rel(h, ref)
    # backward: dU = (dY Wo) through the mask, Wo = [K2, N] k-major operand of the dgrad
    K2 = 256
    dy = torch.randn(M, K2, device=DEV).to(torch.bfloat16)
    wo = (torch.randn(K2, N, device=DEV) * K2 ** -0.5).to(torch.bfloat16)
    du = C.gemm_w4(dy, wo, True, None, None, False, -1, True, 7, p, seed, mask)
    live = (h.float() > 0)  # the mask's meaning: kept and positive
    ref_du = (dy.float() @ wo.float()) * live / (1 - p)
    assert _rel(du, ref_du) < 8e-3, _rel(du, ref_du)
    # bits agree with H wherever H is clearly away from 0 (bf16 rounding of tiny positives aside)
    far = h.float().abs() > 1e-2
    assert torch.equal((du.float() != 0)[far], live[far] & ((dy.float() @ wo.float()) != 0)[far])


@pytest.mark.parametrize("M,K,N", [(512, 256, 512), (2048, 768, 3072), (1280, 256, 1024)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gemm_w4_drelu_from_pingpong_mask(M, K, N, p):
    """The ReLU backward on w4 reading the mask written by csrc/gemm_fused.hip's ping-pong ReLU forward (its thread
    layout, mask_pp) == the ping-pong ReLU backward on the same mask (ops/ffn.py default backward)."""
    C = _ext.native()
    if C.gemm_fused_variant(K) not in (8, 9):
        pytest.skip("ping-pong kernel not chosen for this K")
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    wi = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    mask = torch.zeros(M * N // 32, device=DEV, dtype=torch.int32)
    h = C.gemm_fused(x, wi, False, 1, None, None, None, p, 77, -1, mask)
    dy = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    wo = (torch.randn(K, N, device=DEV) * K ** -0.5).to(torch.bfloat16)
    ref = C.gemm_fused(dy, wo, True, 7, None, None, None, p, 77, -1, mask)
    got = C.gemm_w4(dy, wo, True, None, None, False, -1, True, 7, p, 77, mask, True)
    assert _rel(got, ref) < 1e-3, _rel(got, ref)
    exact = (dy.float() @ wo.float()) * (h.float() > 0) / (1 - p)
    assert _rel(got, exact) < 8e-3


def _gelu_pair_ref(u):
    """fp32 GELU (erf) and its derivative."""
    cdf = 0.5 * (1.0 + torch.erf(u * 0.7071067811865476))
    return u * cdf, cdf + u * 0.3989422804014327 * torch.exp(-0.5 * u * u)


@pytest.mark.parametrize("M,K,N,p,bias", [(8448, 1024, 4096, 0.0, True), (8448, 1024, 4096, 0.1, True),
                                          (1000, 256, 520, 0.0, False), (300, 128, 264, 0.1, True)])
def test_gemm_w4_gelu_forward(M, K, N, p, bias):
    """W4_EPI_GELU: h = s gelu(x wᵀ + b) and aux = s gelu'(.) (s = dropout keep / (1 - p)) vs the fp32 composite with
    the same keep bits (the row-Weyl decisions, ops/rng.py rowwise_keep_mask); persistent (528 tiles) and ragged shapes;
    equal to the ping-pong kernel's epilogue 2 where that kernel runs (M % 256 == 0, N % 256 == 0)."""
    from distributed_llms_example_amd.ops.rng import rowwise_keep_mask
    C = _ext.native()
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    b = (0.5 * torch.randn(N, device=DEV)).to(torch.bfloat16) if bias else None
    aux = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    h = C.gemm_w4(x, w, False, b, None, False, -1, True, 11, p, 31, None, False, None, aux)
    u = x.float() @ w.float().t() + (b.float() if bias else 0.0)
    g, dg = _gelu_pair_ref(u)
    if p > 0:
        keep = rowwise_keep_mask(31, p, M, N, x.device).float() / (1.0 - p)
        g, dg = g * keep, dg * keep
    assert _rel(h, g) < 1e-2, _rel(h, g)
    assert _rel(aux, dg) < 1e-2, _rel(aux, dg)
    if M % 256 == 0 and N % 256 == 0 and bias:
        aux_pp = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        h_pp = C.gemm_fused(x, w, False, 2, b, None, aux_pp, p, 31, 9)
        assert _rel(h, h_pp) < 2e-3 and _rel(aux, aux_pp) < 2e-3, (_rel(h, h_pp), _rel(aux, aux_pp))


@pytest.mark.parametrize("M,d,F_", [(8448, 1024, 4096), (768, 512, 1024), (384, 256, 520)])
def test_gemm_w4_gelu_backward_colsum(M, d, F_):
    """W4_EPI_DGELU: dU = (dY · wo) * aux with per-128-row column sums of dU (the fc1 bias gradient) vs fp32."""
    C = _ext.native()
    torch.manual_seed(M + F_)
    dy = torch.randn(M, d, device=DEV).to(torch.bfloat16)
    wo = (torch.randn(d, F_, device=DEV) * d ** -0.5).to(torch.bfloat16)
    aux = torch.rand(M, F_, device=DEV).to(torch.bfloat16)
    part = torch.full((M // 128, F_), float("nan"), device=DEV)
    du = C.gemm_w4(dy, wo, True, None, None, False, -1, False, 12, 0.0, 0, None, False, aux, None, part)
    ref = (dy.float() @ wo.float()) * aux.float()
    assert _rel(du, ref) < 1e-2, _rel(du, ref)
    ref_part = ref.view(M // 128, 128, F_).sum(1)
    assert _rel(part, ref_part) < 1e-2, _rel(part, ref_part)


@pytest.mark.parametrize("N_out,K_in,M,routed", [(768, 768, 65536, True), (2304, 768, 131072, True),
                                                 (768, 768, 8192, False), (1024, 1024, 65536, True),
                                                 (3072, 1024, 131072, True), (3072, 768, 65536, True)])
def test_default_dgrad_routing(N_out, K_in, M, routed):
    """Default route (ops/routing.py proj_dgrad = rows): a projection's input gradient dX = dY W runs on gemm_w4 from 64K
    token rows at any width and depth (the early-release schedule beats hipBLASLt on every such shape,
    profiles/r6_w4_early_release_ab.txt), on hipBLASLt for micro-batches, and the forward always on hipBLASLt; either way
    it matches fp32."""
    from distributed_llms_example_amd.ops import gemm, routing
    if any(k.startswith("proj_") for k in routing.overrides()):
        pytest.skip(f"DLLM_ROUTE={routing.overrides()} set in the environment")
    torch.manual_seed(N_out + K_in)
    dy = torch.randn(M, N_out, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N_out, K_in, device=DEV) * N_out ** -0.5).to(torch.bfloat16)
    before = gemm.w4_calls
    got = gemm.linear_dgrad(dy, w)
    assert (gemm.w4_calls - before == 1) == routed
    assert _rel(got, dy.float() @ w.float()) < 8e-3
    x = torch.randn(M, K_in, device=DEV).to(torch.bfloat16)
    before = gemm.w4_calls
    gemm.linear_fwd(x, w)
    assert gemm.w4_calls == before  # forwards stay on hipBLASLt
