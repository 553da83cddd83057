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
