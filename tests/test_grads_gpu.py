"""Gradient-path kernels and fp32 gradient accumulation on the GPU.

* wgrad GEMM writing an fp32 flat-buffer slice, ragged M (vocab-sized LM-head gradients);
* native embedding backward (sorted segment-sum) vs ATen, padding_idx, skewed ids, bitwise determinism;
* AdamW with bf16 params and fp32 gradients vs the torch reference step;
* 16-micro-batch gradient accumulation of a bf16 model into the fp32 flat buffer vs the fp64 sum of the
  micro-batches' gradients (accumulation exactness) and vs the fp32 reference model (end-to-end numerics);
* the GA normalisation by the global non-ignored token count.
"""
import os

import pytest
import torch

from distributed_llms_example_amd import _ext
from distributed_llms_example_amd.models import build_model, resolve_config

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


@pytest.mark.parametrize("K,M,N,beta,splits", [
    (4096, 32128 // 4, 768, True, 0),  # ragged last M tile (8032 = 31 x 256 + 96), fp32 accumulate
    (1024, 1000, 512, False, 1),       # ragged M, direct (unsplit) fp32 epilogue
    (4096, 768, 768, True, 0),         # t5-base o-proj class
    (2048, 264, 256, True, 3),         # two M tiles, the second 8 rows tall
])
def test_gemm_wgrad_fp32_out_ragged_m(K, M, N, beta, splits):
    """csrc/gemm_w4.hip weight-gradient mode (the only wgrad kernel since round 6), fp32 output vs fp64."""
    torch.manual_seed(0)
    a = torch.randn(K, M, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
    c0 = torch.randn(M, N, device=DEV, dtype=torch.float32)
    c = c0.clone()
    C = _ext.native()
    assert C.gemm_wgrad_supported(a, b, c)
    C.gemm_wgrad(a, b, c, beta, -1, splits)
    ref = a.double().t() @ b.double() + (c0.double() if beta else 0)
    assert _rel(c, ref) < 1e-5, _rel(c, ref)


@pytest.mark.parametrize("splits", [0, 1])
def test_gemm_wgrad_ragged_m_bf16_out_and_no_overrun(splits):
    """bf16 output, ragged M: rows past M are never written (guard row below the output stays intact)."""
    torch.manual_seed(1)
    K, M, N = 2048, 520, 256
    a = torch.randn(K, M, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
    big = torch.full((M + 8, N), 7.0, device=DEV, dtype=torch.bfloat16)
    c = big[:M]
    _ext.native().gemm_wgrad(a, b, c, False, -1, splits)
    ref = a.float().t() @ b.float()
    assert _rel(c, ref) < 5e-3
    assert bool((big[M:] == 7.0).all())


@pytest.mark.parametrize("splits", [0, 1, 5])
def test_gemm_wgrad_w4_strided_operands(splits):
    """w4 weight-gradient mode on strided [K, M] / [K, N] views whose gaps hold NaN: the k-major images' column overrun
    (past M in the last row tile) reads the gap, which may only reach output rows >= M — never stored; fp32 and bf16
    accumulate (beta) agree with the fp64 product."""
    torch.manual_seed(2)
    K, M, N = 3072, 520, 512
    af = torch.full((K, M + 72), float("nan"), device=DEV, dtype=torch.bfloat16)
    bf = torch.full((K, N + 64), float("nan"), device=DEV, dtype=torch.bfloat16)
    a, b = af[:, :M], bf[:, :N]
    a.copy_(torch.randn(K, M, device=DEV))
    b.copy_(torch.randn(K, N, device=DEV))
    ref = a.double().t() @ b.double()
    C = _ext.native()
    for dt, tol in ((torch.float32, 1e-5), (torch.bfloat16, 5e-3)):
        c0 = torch.randn(M, N, device=DEV).to(dt)
        c = c0.clone()
        C.gemm_wgrad(a, b, c, True, 12, splits)
        assert _rel(c, ref + c0.double()) < tol, (dt, _rel(c, ref + c0.double()))


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("pad", [None, 1])
def test_embed_bwd_matches_aten(out_dtype, pad):
    torch.manual_seed(0)
    V, d, T = 5000, 768, 40000
    ids = torch.randint(0, V, (T,), device=DEV)
    ids[::3] = 1                     # one id with ~13K rows (padding-like skew: runs over many windows)
    ids[5:200] = 4999                # a long contiguous run
    dy = torch.randn(T, d, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(V, d, device=DEV, requires_grad=True)
    torch.nn.functional.embedding(ids, w, padding_idx=pad).backward(dy.float())
    ref = w.grad.double()
    srt, perm = torch.sort(ids, stable=True)
    outs = []
    for _ in range(2):
        out = torch.zeros(V, d, device=DEV, dtype=out_dtype)
        _ext.native().embed_bwd(srt, perm, dy, out, -1 if pad is None else pad)
        outs.append(out)
    tol = 1e-6 if out_dtype == torch.float32 else 5e-3
    assert _rel(outs[0], ref) < tol, _rel(outs[0], ref)
    assert torch.equal(outs[0], outs[1]), "embedding backward must be deterministic"
    if pad is not None:
        assert bool((outs[0][pad] == 0).all())


def test_embedding_op_accumulates_into_flat_buffer():
    from distributed_llms_example_amd.ops.embedding import embedding
    from distributed_llms_example_amd.parallel.flat import FlatParams
    emb = torch.nn.Embedding(1000, 256).cuda().to(torch.bfloat16)
    flat = FlatParams(emb, grad_dtype=torch.float32)
    ids = torch.randint(0, 1000, (4, 300), device=DEV)
    g = torch.randn(4, 300, 256, device=DEV, dtype=torch.bfloat16)
    for _ in range(2):
        embedding(ids, emb.weight).backward(g)
    ref = torch.zeros(1000, 256, device=DEV, dtype=torch.float64).index_add_(0, ids.flatten(),
                                                                           g.reshape(-1, 256).double())
    assert emb.weight.grad is None  # fp32 gradients live in the flat buffer only
    assert _rel(flat.grad_view(0), 2 * ref) < 1e-6


def test_adamw_bf16_params_fp32_grads():
    from distributed_llms_example_amd.ops.optim import FusedAdamW
    from distributed_llms_example_amd.parallel.flat import FlatParams
    torch.manual_seed(0)
    m = torch.nn.Linear(512, 384).cuda().to(torch.bfloat16)
    flat = FlatParams(m, grad_dtype=torch.float32)
    opt = FusedAdamW(flat, lr=1e-3, weight_decay=0.01)
    ref_p = flat.param_buf.float().clone()
    ref_m = torch.zeros_like(ref_p)
    ref_v = torch.zeros_like(ref_p)
    for step in range(1, 4):
        flat.grad_buf.copy_(torch.randn_like(flat.grad_buf) * 1e-3)  # tiny values: bf16 would lose them
        g = flat.grad_buf.clone()
        opt.step(max_grad_norm=None)
        ref_p.mul_(1 - 1e-3 * 0.01)
        ref_m.lerp_(g, 0.1)
        ref_v.mul_(0.999).addcmul_(g, g, value=0.001)
        denom = (ref_v.sqrt() / (1 - 0.999 ** step) ** 0.5).add_(1e-8)
        ref_p.addcdiv_(ref_m, denom, value=-1e-3 / (1 - 0.9 ** step))
        assert _rel(opt.master, ref_p) < 1e-6
        assert _rel(flat.param_buf, ref_p) < 5e-3


def _small_cfg():
    c = resolve_config("t5-base")
    return c.replace(num_layers=2, num_decoder_layers=2, vocab_size=4096, d_model=512, num_heads=8, d_kv=64,
                     d_ff=1024, dropout_rate=0.0, attention_dropout=0.0)


def _micro_batches(cfg, n=16, B=2, S=256, T=64, ignore=False):
    g = torch.Generator().manual_seed(3)
    out = []
    for i in range(n):
        ids = torch.randint(3, cfg.vocab_size, (B, S), generator=g)
        am = torch.ones(B, S, dtype=torch.long)
        am[1, S - 17 * (i % 4):] = 0
        lab = torch.randint(3, cfg.vocab_size, (B, T), generator=g)
        if ignore:  # very different numbers of ignored targets per micro-batch (1..61 + 10 or 64 kept)
            lab[0, 1 + 20 * (i % 4):] = -100
            if i % 2 == 0:
                lab[1, 10:] = -100
        out.append({k: v.cuda() for k, v in dict(input_ids=ids, attention_mask=am, labels=lab).items()})
    return out


def _engine(cfg, sd, grad_dtype):
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.engine import TrainEngine
    m = build_model(cfg)
    m.load_state_dict(sd)
    eng = TrainEngine(m, init_distributed(), lr=1e-4, dtype=torch.bfloat16, grad_dtype=grad_dtype)
    eng.train()
    return eng


def test_ga16_fp32_accumulation_matches_fp64_sum_and_fp32_reference():
    cfg = _small_cfg()
    torch.manual_seed(0)
    sd = build_model(cfg).state_dict()
    mbs = _micro_batches(cfg)
    ga = len(mbs)
    eng = _engine(cfg, sd, torch.float32)
    assert eng.flat.grad_buf.dtype == torch.float32
    # fp64 sum of each micro-batch's own gradient (each computed alone into a zeroed fp32 buffer)
    acc = torch.zeros(eng.flat.numel, dtype=torch.float64, device=DEV)
    for b in mbs:
        eng.optimizer.zero_grad()
        eng.forward_backward(b, grad_accum=ga)
        acc += eng.flat.grad_buf.double()
    eng.optimizer.zero_grad()
    for i, b in enumerate(mbs):
        eng.forward_backward(b, grad_accum=ga, sync=i + 1 == ga)
    g32 = eng.flat.grad_buf.double().clone()
    assert _rel(g32, acc) < 2e-6, _rel(g32, acc)
    # the bf16 buffer (DLLM_GRAD_DTYPE=bf16) rounds every one of the 16 adds: measurably worse
    e16 = _engine(cfg, sd, torch.bfloat16)
    for i, b in enumerate(mbs):
        e16.forward_backward(b, grad_accum=ga, sync=i + 1 == ga)
    err16 = _rel(e16.flat.grad_buf, acc)
    assert err16 > 10 * _rel(g32, acc), err16
    # end to end vs the fp32 reference model on the whole batch (torch reference ops, fp32 weights)
    m32 = build_model(cfg).cuda()
    m32.load_state_dict(sd)
    m32.train()
    os.environ["DLLM_REFERENCE_OPS"] = "1"
    try:
        for b in mbs:
            (m32(**b).loss / ga).backward()
    finally:
        os.environ.pop("DLLM_REFERENCE_OPS")
    worst = 1.0
    for seg, p32 in zip(eng.flat.segments, [dict(m32.named_parameters())[s.name] for s in eng.flat.segments]):
        g = g32[seg.offset:seg.offset + seg.numel]
        r = p32.grad.double().flatten()
        if r.norm() == 0:
            continue
        worst = min(worst, torch.nn.functional.cosine_similarity(g, r, dim=0).item())
    assert worst > 0.995, worst


def test_global_token_normalisation_equals_full_batch_mean():
    """forward_backward(num_items=N) over micro-batches with different ignored-token counts == the gradient of the
    mean over ALL non-ignored tokens of the step, not the mean of micro-batch means."""
    from distributed_llms_example_amd.train.engine import token_count
    cfg = _small_cfg()
    torch.manual_seed(0)
    sd = build_model(cfg).state_dict()
    mbs = _micro_batches(cfg, n=4, ignore=True)
    eng = _engine(cfg, sd, torch.float32)
    n = sum(token_count(b["labels"]) for b in mbs)
    for i, b in enumerate(mbs):
        eng.forward_backward(b, sync=i + 1 == len(mbs), num_items=n)
    g = eng.flat.grad_buf.double().clone()
    # reference: one batch holding all micro-batches (the CE mean then runs over all non-ignored tokens)
    full = {k: torch.cat([b[k] for b in mbs]) for k in mbs[0]}
    ref_eng = _engine(cfg, sd, torch.float32)
    ref_eng.forward_backward(full)
    assert _rel(g, ref_eng.flat.grad_buf) < 2e-2, _rel(g, ref_eng.flat.grad_buf)
    # the per-micro-batch-mean normalisation differs measurably here
    alt = _engine(cfg, sd, torch.float32)
    for i, b in enumerate(mbs):
        alt.forward_backward(b, grad_accum=len(mbs), sync=i + 1 == len(mbs))
    assert _rel(alt.flat.grad_buf, ref_eng.flat.grad_buf) > 3 * _rel(g, ref_eng.flat.grad_buf)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("bias,smooth,V", [(False, 0.0, 32128), (True, 0.1, 50265), (False, 0.1, 4000)])
def test_lm_head_chunked_ce_matches_fp32(bias, smooth, V, fused, monkeypatch):
    """LM head + CE without materialised logits (ops/lm_head.py) vs F.cross_entropy on fp32 logits: loss, dh, dW (flat
    buffer).  fused=1: CE inside the GEMM epilogues (csrc/gemm_w4.hip CEF / CEB + csrc/ce.hip merge); 0: vocab chunks."""
    from distributed_llms_example_amd.ops import lm_head as LH
    from distributed_llms_example_amd.ops.lm_head import lm_head_loss
    from distributed_llms_example_amd.parallel.flat import FlatParams
    # several chunks, ragged last one; fused "1": the GEMM-epilogue CE, "0": vocabulary chunks
    monkeypatch.setenv("DLLM_ROUTE", "lmhead_chunk_mb=8,lmhead=" + ("fused" if fused == "1" else "logits"))
    torch.manual_seed(0)
    N, d = 1000, 768
    emb = torch.nn.Embedding(V, d).cuda().to(torch.bfloat16)
    with torch.no_grad():
        emb.weight.normal_(0, 0.05)
    flat = FlatParams(emb, grad_dtype=torch.float32)
    h = (torch.randn(N, d, device=DEV) * 0.5).to(torch.bfloat16).requires_grad_(True)
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::7] = -100
    b = (torch.randn(V, device=DEV) * 0.1) if bias else None
    calls = []
    if fused == "1":  # the GEMM-epilogue path must be the one that runs
        real = LH._LMHeadCEFusedFn.apply
        monkeypatch.setattr(LH._LMHeadCEFusedFn, "apply", lambda *a: (calls.append(1), real(*a))[1])
    loss = lm_head_loss(h, emb.weight, labels, scale=0.5, bias=b, label_smoothing=smooth)
    loss.backward()
    assert calls == ([1] if fused == "1" else [])
    hr = h.detach().float().requires_grad_(True)
    wr = emb.weight.detach().float().requires_grad_(True)
    logits = (hr * 0.5) @ wr.t() + (b if bias else 0)
    ref = torch.nn.functional.cross_entropy(logits, labels, ignore_index=-100, label_smoothing=smooth)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 2e-3 * ref.item(), (loss.item(), ref.item())
    assert _rel(h.grad, hr.grad) < 1e-2, _rel(h.grad, hr.grad)
    assert _rel(flat.grad_view(0), wr.grad) < 1e-2, _rel(flat.grad_view(0), wr.grad)


@pytest.mark.parametrize("V", [32128, 50265, 4000, 128112])
def test_lm_head_fused_lse_exact(V):
    """The GEMM-epilogue CE forward's per-row lse / loss vs fp32 logsumexp on the same bf16 operands, at fp32-rounding
    tolerance.  ceil(V / 128) odd (T5 32128, BART 50265, M2M100 128112) is the case where a tile's second 128-column
    half lies wholly past V: its partial must not be written (it would land in the next row's first slot and drop
    vocabulary columns 0..127 from that row).  Columns 0..127 carry most of the mass here, so a dropped slot moves lse
    by O(1); near-uniform logits would hide it (4e-4 relative)."""
    C = _ext.native()
    torch.manual_seed(1)
    N, d = 777, 256
    h = (torch.randn(N, d, device=DEV) * 0.5).to(torch.bfloat16)
    w = (torch.randn(V, d, device=DEV) * 0.1).to(torch.bfloat16)
    bias = torch.zeros(V, device=DEV)
    bias[:128] = 4.0
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::5] = -100
    labels[1::5] = 3
    ref = torch.logsumexp(h.float() @ w.float().t() + bias, dim=1)
    for _ in range(3):
        loss_rows, lse = C.lmhead_ce_fwd(h, w, labels, bias, 0.0, -100)
        torch.cuda.synchronize()
        assert (lse - ref).abs().max().item() < 2e-4 * ref.abs().max().item(), (lse - ref).abs().max().item()
        lg = h.float() @ w.float().t() + bias
        valid = labels != -100
        ref_loss = torch.nn.functional.cross_entropy(lg[valid], labels[valid], reduction="none")
        assert (loss_rows[valid] - ref_loss).abs().max().item() < 1e-3, (loss_rows[valid] - ref_loss).abs().max().item()


def test_t5_chunked_lm_head_matches_full(monkeypatch):
    """The T5 model's loss / flat gradient with the chunked LM head == with materialised logits."""
    cfg = _small_cfg()
    torch.manual_seed(0)
    sd = build_model(cfg).state_dict()
    b = _micro_batches(cfg, n=1, B=4)[0]
    res = []
    for full_mb in ("-1", "0"):  # this test pins the vocab-chunked path against full logits
        monkeypatch.setenv("DLLM_ROUTE", f"lmhead=logits,lmhead_full_mb={full_mb}")
        eng = _engine(cfg, sd, torch.float32)
        loss = eng.forward_backward(b)
        res.append((float(loss), eng.flat.grad_buf.clone()))
    assert abs(res[0][0] - res[1][0]) < 1e-3 * res[0][0]
    assert _rel(res[1][1], res[0][1]) < 1e-2, _rel(res[1][1], res[0][1])


def test_t5_fused_lm_head_matches_materialised_logits(monkeypatch):
    """bf16 T5: the loss / flat gradient with the GEMM-epilogue CE == with materialised bf16 logits + the CE kernels
    (fp32 logits inside the epilogue vs bf16-rounded ones: bf16-noise agreement)."""
    cfg = _small_cfg()
    torch.manual_seed(0)
    sd = build_model(cfg).state_dict()
    b = _micro_batches(cfg, n=1, B=4)[0]
    res = []
    for fused in ("1", "0"):  # never chunked: "1" forces the fused path, "0" full logits
        monkeypatch.setenv("DLLM_ROUTE", "lmhead_full_mb=-1,lmhead=" + ("fused" if fused == "1" else "logits"))
        eng = _engine(cfg, sd, torch.float32)
        eng.train(False)
        loss = eng.forward_backward(b)
        res.append((float(loss), eng.flat.grad_buf.float().clone()))
    assert abs(res[0][0] - res[1][0]) < 5e-3 * res[1][0], (res[0][0], res[1][0])
    assert _rel(res[0][1], res[1][1]) < 3e-2, _rel(res[0][1], res[1][1])


@pytest.mark.parametrize("graphed", [False, True])
@pytest.mark.parametrize("sites", [None, "qkv,wi,o"])
def test_side_stream_wgrad_matches_single_stream(graphed, sites, monkeypatch):
    """Weight gradients on the side stream (ops/streams.py) == all on the compute stream: same flat gradient (the
    kernels are deterministic and the accumulation order is unchanged), eager and inside a captured HIP graph; the side
    path really ran.  ``sites``: the paired mode (only those layers' weight gradients, joined at the next norm /
    attention backward)."""
    from distributed_llms_example_amd.ops import streams
    monkeypatch.setattr(streams, "SITES", frozenset(sites.split(",")) if sites else None)
    cfg = _small_cfg().replace(dropout_rate=0.0)
    torch.manual_seed(0)
    sd = build_model(cfg).state_dict()
    mbs = _micro_batches(cfg, n=2, B=2)
    res = []
    for on in ("1", "0"):  # "1": forced on (the default "auto" enables it for small micro-batches only)
        monkeypatch.setenv("DLLM_ROUTE", f"wgrad_stream={on}")
        eng = _engine(cfg, sd, torch.float32)
        eng.train(False)
        n0 = streams.launches
        if graphed:
            from distributed_llms_example_amd.train.graph import GraphedStep
            gs = GraphedStep(eng, mbs, warmup=1)
            gs.replay(mbs)
            eng.disable_step_seeds()
            # the step ends with AdamW (reading every gradient) and zero_grad: the parameters after two optimizer steps
            # (warmup + replay) carry the gradients; they must match the single-stream run bit for bit
            res.append((float(gs.loss), eng.flat.param_buf.float().clone(), streams.launches - n0))
        else:
            for i, b in enumerate(mbs):
                eng.forward_backward(b, grad_accum=len(mbs), sync=i + 1 == len(mbs))
            torch.cuda.synchronize()
            res.append((0.0, eng.flat.grad_buf.float().clone(), streams.launches - n0))
    (l1, g1, n1), (l0, g0, n0) = res
    assert n1 > 0 and n0 == 0, (n1, n0)
    assert l1 == l0
    assert torch.equal(g1, g0), _rel(g1, g0)


@pytest.mark.parametrize("sq_force", ["0", "1"])
def test_bart_attention_bias_colsum_matches_column_reduction(sq_force, monkeypatch):
    """BART: the q / k / v projection bias gradients summed by the attention backward kernels (dQ / dK / dV epilogues,
    csrc/attn.hip cs_wave) == a separate column reduction of the same dQKV (ops/attention.py BIAS_COLSUM off), with
    ragged sequence lengths (partial last blocks) and both cross-attention dK/dV kernels (``sq_force``: the
    short-query kernel forced on); every other gradient is unchanged bit for bit; the hand-off really ran."""
    from distributed_llms_example_amd.ops import attention as A
    from distributed_llms_example_amd.ops import gemm as G
    from distributed_llms_example_amd.ops.linear import _gbuf
    monkeypatch.setenv("DLLM_ROUTE", f"attn_dkdv_sq_force={sq_force}")
    cfg = resolve_config("bart-large").replace(num_layers=2, num_decoder_layers=2, vocab_size=4096, d_model=512,
                                               num_heads=8, d_ff=1024, dropout_rate=0.0, attention_dropout=0.0)
    torch.manual_seed(0)
    sd = build_model(cfg).state_dict()
    b = _micro_batches(cfg, n=1, B=3, S=200, T=72)[0]
    res = []
    for on in (True, False):
        monkeypatch.setattr(A, "BIAS_COLSUM", on)
        eng = _engine(cfg, sd, torch.float32)
        eng.train(False)
        n0 = G.colsum_handoffs
        eng.forward_backward(b)
        torch.cuda.synchronize()
        bias = {n: _gbuf(p).float().clone() for n, p in eng.model.named_parameters()
                if n.endswith(("qkv_proj.bias", "q_proj.bias", "kv_proj.bias"))}
        res.append((eng.flat.grad_buf.float().clone(), bias, G.colsum_handoffs - n0))
    (g1, b1, h1), (g0, b0, h0) = res
    assert len(b1) == 2 + 2 * 3, sorted(b1)  # encoder qkv x2, decoder qkv / q / kv x2
    # 4 self-attention qkv + 2 cross q + 2 cross kv sums on top of the post-LN hand-offs both runs share
    assert h1 - h0 == 8, (h1, h0)
    for n in b1:
        assert _rel(b1[n], b0[n]) < 1e-5, (n, _rel(b1[n], b0[n]))
    mask = torch.ones_like(g1, dtype=torch.bool)
    for n, p in eng.model.named_parameters():
        if n in b1:
            gb = _gbuf(p)
            off = (gb.data_ptr() - eng.flat.grad_buf.data_ptr()) // gb.element_size()
            mask[off:off + gb.numel()] = False
    assert torch.equal(g1[mask], g0[mask])


def test_gemm_wgrad_w4_wide_leading_dim():
    """A [K, M] view of a 40000-column buffer with one split requested: its k-rows span > 4 GB, past one buffer
    descriptor's 32-bit range — the binding raises the split count until each split's span fits (csrc/bind.cpp)."""
    torch.manual_seed(3)
    K, M, N, LD = 65536, 256, 256, 40000
    af = torch.empty(K, LD, device=DEV, dtype=torch.bfloat16)
    a = af[:, :M]
    a.copy_(torch.randn(K, M, device=DEV))
    b = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
    c = torch.zeros(M, N, device=DEV, dtype=torch.float32)
    splits = _ext.native().gemm_wgrad(a, b, c, True, 12, 1)
    assert splits >= 2, splits
    ref = a.double().t() @ b.double()
    assert _rel(c, ref) < 1e-5, _rel(c, ref)


@pytest.mark.parametrize("model", ["t5", "bart"])
def test_deferred_weight_gradients_gpu(model, monkeypatch):
    """bf16 on the GPU, side streams on: GA 4 with the weight gradients deferred to the window's last micro-batch (one
    w4 weight-gradient GEMM over the concatenated tokens) == per-micro-batch GEMMs, up to fp32 summation order."""
    cfg = _small_cfg()
    if model == "bart":
        cfg = resolve_config("bart-large").replace(num_layers=2, num_decoder_layers=2, vocab_size=4096, d_model=512,
                                                   num_heads=8, d_ff=1024, dropout_rate=0.0, attention_dropout=0.0)
    torch.manual_seed(0)
    sd = build_model(cfg).state_dict()
    mbs = _micro_batches(cfg, n=4, B=2)
    res = []
    for mode in ("1", "0"):
        monkeypatch.setenv("DLLM_DEFER_WGRAD", mode)
        monkeypatch.setenv("DLLM_ROUTE", "wgrad_stream=1")
        eng = _engine(cfg, sd, torch.float32)
        eng.train(False)
        for i, b in enumerate(mbs):
            eng.forward_backward(b, grad_accum=4, sync=i == 3)
        torch.cuda.synchronize()
        res.append((eng.flat.grad_buf.float().clone(), eng.wgrad_defer.merged))
    (g1, m1), (g0, m0) = res
    assert m1 > 0 and m0 == 0
    assert _rel(g1, g0) < 1e-5, _rel(g1, g0)


@pytest.mark.parametrize("nseg,rows,M,N", [(5, 1024, 520, 512), (16, 192, 768, 768), (32, 64, 256, 256)])
def test_gemm_wgrad_segs_matches_fp64(nseg, rows, M, N):
    """The w4 weight-gradient mode over deferred micro-batch segments read in place (csrc/bind.cpp gemm_wgrad_segs):
    Σ_i a_iᵀ b_i + C for fp32 / bf16 C, ragged M, strided segments."""
    torch.manual_seed(4)
    af = torch.randn(nseg, rows, M + 8, device=DEV, dtype=torch.bfloat16)
    bs = [torch.randn(rows, N, device=DEV, dtype=torch.bfloat16) for _ in range(nseg)]
    as_ = [af[i, :, :M] for i in range(nseg)]
    ref = sum(a.double().t() @ b.double() for a, b in zip(as_, bs))
    C = _ext.native()
    for dt, tol in ((torch.float32, 1e-5), (torch.bfloat16, 5e-3)):
        c0 = torch.randn(M, N, device=DEV).to(dt)
        c = c0.clone()
        C.gemm_wgrad_segs(as_, bs, c, True)
        assert _rel(c, ref + c0.double()) < tol, (dt, _rel(c, ref + c0.double()))
