"""Context-parallel ring attention (parallel/context.py) on CPU/gloo: the sharded op must equal the unsharded
attention (T5 relative bias by global distance, key padding) in forward and in every gradient, including the
bucket table's."""
import pytest
import torch
import torch.distributed as dist

from test_distributed_cpu import run_ranks


def _inputs(B=2, S=24, H=3, D=8, seed=0):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(B, S, H, D, generator=g)
    k = torch.randn(B, S, H, D, generator=g)
    v = torch.randn(B, S, H, D, generator=g)
    table = torch.randn(32, H, generator=g)
    do = torch.randn(B, S, H, D, generator=g)
    kpm = torch.ones(B, S, dtype=torch.bool)
    kpm[1, S - 5:] = False  # padded tail (lands on the last shard)
    return q, k, v, table, do, kpm


def _full(q, k, v, table, do, kpm, scale):
    from distributed_llms_example_amd.ops.attention import _reference, relative_bias_lut
    q, k, v, table = (t.clone().requires_grad_(True) for t in (q, k, v, table))
    S = q.shape[1]
    lut = relative_bias_lut(table, S, S, True, 32, 128)
    o = _reference(q, k, v, scale, False, kpm, lut, 0.0, 0)
    o.backward(do)
    return o.detach(), q.grad, k.grad, v.grad, table.grad


def _ring_case(rank, world, scale=1.0, use_bias=True, use_kpm=True, S=24):
    from distributed_llms_example_amd.parallel.context import ring_attention
    q, k, v, table, do, kpm = _inputs(S=S)
    s = S // world
    sl = slice(rank * s, rank * s + s)
    ql, kl, vl = (t[:, sl].clone().requires_grad_(True) for t in (q, k, v))
    tab = table.clone().requires_grad_(True)
    o = ring_attention(ql, kl, vl, scale=scale, key_padding_mask=kpm[:, sl] if use_kpm else None,
                       bias_table=tab if use_bias else None)
    o.backward(do[:, sl])
    gt = tab.grad if use_bias else torch.zeros(1)
    dist.all_reduce(gt)  # table gradient = sum of the ranks' partial sums (what the DP x CP reducer does)
    return o.detach(), ql.grad, kl.grad, vl.grad, gt


@pytest.mark.parametrize("world", [2, 3])
def test_ring_attention_matches_full(world):
    import functools
    out = run_ranks(functools.partial(_ring_case, S=24), world=world)
    q, k, v, table, do, kpm = _inputs(S=24)
    o, dq, dk, dv, dt = _full(q, k, v, table, do, kpm, 1.0)
    s = 24 // world
    for r in range(world):
        sl = slice(r * s, r * s + s)
        ro, rdq, rdk, rdv, rdt = (torch.as_tensor(x) for x in out[r])
        torch.testing.assert_close(ro, o[:, sl], atol=2e-5, rtol=1e-4)
        torch.testing.assert_close(rdq, dq[:, sl], atol=2e-5, rtol=1e-4)
        torch.testing.assert_close(rdk, dk[:, sl], atol=2e-5, rtol=1e-4)
        torch.testing.assert_close(rdv, dv[:, sl], atol=2e-5, rtol=1e-4)
        torch.testing.assert_close(rdt, dt, atol=1e-4, rtol=1e-4)


def test_ring_attention_bart_style_no_bias():
    import functools
    out = run_ranks(functools.partial(_ring_case, scale=8 ** -0.5, use_bias=False), world=2)
    q, k, v, table, do, kpm = _inputs()
    from distributed_llms_example_amd.ops.attention import _reference
    qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v))
    o = _reference(qq, kk, vv, 8 ** -0.5, False, kpm, None, 0.0, 0)
    o.backward(do)
    for r in range(2):
        sl = slice(r * 12, r * 12 + 12)
        ro, rdq, rdk, rdv, _ = (torch.as_tensor(x) for x in out[r])
        torch.testing.assert_close(ro, o.detach()[:, sl], atol=2e-5, rtol=1e-4)
        torch.testing.assert_close(rdk, kk.grad[:, sl], atol=2e-5, rtol=1e-4)
        torch.testing.assert_close(rdv, vv.grad[:, sl], atol=2e-5, rtol=1e-4)


def test_merge_and_block_math_single_process():
    """W=1 path (no process group) equals the reference op; block merge of two halves equals the whole."""
    from distributed_llms_example_amd.parallel import context as cp
    q, k, v, table, do, kpm = _inputs(S=16)
    o_all, lse_all = cp._ref_block_fwd(q, k, v, kpm, None, 1.0, 0.0, 0)
    o1, l1 = cp._ref_block_fwd(q, k[:, :8], v[:, :8], kpm[:, :8], None, 1.0, 0.0, 0)
    o2, l2 = cp._ref_block_fwd(q, k[:, 8:], v[:, 8:], kpm[:, 8:], None, 1.0, 0.0, 0)
    om, lm = cp._merge(o1, l1, o2, l2)
    torch.testing.assert_close(om, o_all, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(lm, lse_all, atol=1e-5, rtol=1e-5)
    # a block whose keys are all padded contributes nothing
    kpm0 = kpm.clone()
    kpm0[:, 8:] = False
    o3, l3 = cp._ref_block_fwd(q, k[:, 8:], v[:, 8:], kpm0[:, 8:], None, 1.0, 0.0, 0)
    assert torch.isinf(l3).all()
    om2, lm2 = cp._merge(o1, l1, o3, l3)
    torch.testing.assert_close(om2, o1, atol=1e-6, rtol=1e-6)


def _t5_cp_case(rank, world, name="t5-tiny"):
    from distributed_llms_example_amd.models import build_model
    from distributed_llms_example_amd.parallel.context import shard_sequence
    torch.manual_seed(0)
    model = build_model(name).eval()
    model.enable_context_parallel(None)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(3, 500, (3, 16), generator=g)
    mask = torch.ones(3, 16, dtype=torch.long)
    mask[2, 11:] = 0
    lab = torch.randint(3, 500, (3, 6), generator=g)
    out = model(input_ids=shard_sequence(ids), attention_mask=shard_sequence(mask), labels=lab)
    out.loss.backward()
    grads = []
    for p in model.parameters():  # what the data-parallel reducer does: average over ranks
        gr = p.grad.clone()
        dist.all_reduce(gr)
        grads.append(gr / world)
    return out.loss.detach(), grads


@pytest.mark.parametrize("world,name", [(2, "t5-tiny"), (4, "t5-tiny"), (2, "umt5-tiny")])
def test_t5_context_parallel_matches_single_process(world, name):
    import functools
    from distributed_llms_example_amd.models import build_model
    out = run_ranks(functools.partial(_t5_cp_case, name=name), world=world)
    torch.manual_seed(0)
    model = build_model(name).eval()
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(3, 500, (3, 16), generator=g)
    mask = torch.ones(3, 16, dtype=torch.long)
    mask[2, 11:] = 0
    lab = torch.randint(3, 500, (3, 6), generator=g)
    ref = model(input_ids=ids, attention_mask=mask, labels=lab)
    ref.loss.backward()
    for r in range(world):
        loss, grads = out[r]
        assert float(loss) == pytest.approx(float(ref.loss), rel=1e-5, abs=1e-6)
        for (n, p), gr in zip(model.named_parameters(), grads):
            torch.testing.assert_close(torch.as_tensor(gr), p.grad, atol=1e-5, rtol=1e-4, msg=n)


def test_chunked_attention_matches_full():
    from distributed_llms_example_amd.parallel.context import chunked_attention
    q, k, v, table, do, kpm = _inputs(S=24)
    o, dq, dk, dv, dt = _full(q, k, v, table, do, kpm, 1.0)
    a = [t.clone().requires_grad_(True) for t in (q, k, v, table)]
    oc = chunked_attention(a[0], a[1], a[2], chunk=8, key_padding_mask=kpm, bias_table=a[3])
    oc.backward(do)
    torch.testing.assert_close(oc.detach(), o, atol=2e-5, rtol=1e-4)
    for x, y in zip(a, (dq, dk, dv, dt)):
        torch.testing.assert_close(x.grad, y, atol=5e-5, rtol=1e-4)


@pytest.mark.parametrize("name", ["t5-tiny", "umt5-tiny"])
def test_t5_long_sequence_chunked_encoder(monkeypatch, name):
    """Above ops/routing.py attn_chunk_min tokens the T5 encoder runs chunked attention: same loss and gradients."""
    from distributed_llms_example_amd.models import build_model
    torch.manual_seed(0)
    model = build_model(name).eval()
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(3, 500, (2, 24), generator=g)
    mask = torch.ones(2, 24, dtype=torch.long)
    mask[1, 17:] = 0
    lab = torch.randint(3, 500, (2, 6), generator=g)
    ref = model(input_ids=ids, attention_mask=mask, labels=lab)
    ref.loss.backward()
    g_ref = [p.grad.clone() for p in model.parameters()]
    model.zero_grad(set_to_none=True)
    monkeypatch.setenv("DLLM_ROUTE", "attn_chunk=8,attn_chunk_min=16")
    out = model(input_ids=ids, attention_mask=mask, labels=lab)
    out.loss.backward()
    assert float(out.loss) == pytest.approx(float(ref.loss), rel=1e-5)
    for (n, p), gr in zip(model.named_parameters(), g_ref):
        torch.testing.assert_close(p.grad, gr, atol=1e-5, rtol=1e-4, msg=n)


def test_chunked_attention_ragged_length():
    """A length with no divisor near the chunk (a prime) is padded to whole blocks with masked keys."""
    from distributed_llms_example_amd.parallel.context import chunked_attention
    q, k, v, table, do, kpm = _inputs(S=23)
    o, dq, dk, dv, dt = _full(q, k, v, table, do, kpm, 1.0)
    a = [t.clone().requires_grad_(True) for t in (q, k, v, table)]
    oc = chunked_attention(a[0], a[1], a[2], chunk=8, key_padding_mask=kpm, bias_table=a[3])
    oc.backward(do)
    torch.testing.assert_close(oc.detach(), o, atol=2e-5, rtol=1e-4)
    for x, y in zip(a, (dq, dk, dv, dt)):
        torch.testing.assert_close(x.grad, y, atol=5e-5, rtol=1e-4)


def test_long_sequence_chunk_prime_lengths(monkeypatch):
    from distributed_llms_example_amd.parallel.context import long_sequence_chunk
    monkeypatch.delenv("DLLM_ROUTE", raising=False)
    for n in (9001, 10007, 8200, 16384, 32768, 65521):
        c = long_sequence_chunk(n, rows=64)
        blocks = -(-n // c)
        assert c % 128 == 0 and 2048 <= c <= 4096 + 128 and blocks * c - n < 128 * blocks, (n, c)
    assert long_sequence_chunk(16384, rows=64) == 4096
    assert long_sequence_chunk(32768, rows=12) == 8192
    assert long_sequence_chunk(8192, rows=64) is None
