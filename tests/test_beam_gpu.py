"""csrc/beam.hip (one beam-search step: log_softmax normaliser + processors + beam score + top-2·nb) vs the torch
composite of models/generation.py on the same logits, and whole beam-search generation with the fused step vs the
composite step."""
import pytest
import torch

from distributed_llms_example_amd import _ext
from distributed_llms_example_amd.models import build_model, resolve_config
from distributed_llms_example_amd.models import generation as gen

pytestmark = pytest.mark.gpu


def _composite(logits, beam_scores, seqs, cur, B, nb, proc):
    """All nb·V candidate scores per batch entry and their top-2·nb (torch ops, models/generation.py)."""
    min_length, ngram, fb, fe, max_length, eos = proc
    logp = gen._apply_processors_device(torch.log_softmax(logits.float(), dim=-1), seqs, cur, min_length, ngram, fb,
                                        fe, max_length, eos)
    V = logp.shape[-1]
    cand = (beam_scores.view(-1, 1) + logp).view(B, nb * V)
    return cand, cand.topk(2 * nb, dim=1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("nb", [1, 2, 4])
@pytest.mark.parametrize("case", ["plain", "minlen", "ngram", "force_bos", "force_eos"])
def test_beam_topk_matches_composite(dtype, nb, case):
    torch.manual_seed(0)
    B, V, L = 37, 50265, 40
    cur = 1 if case == "force_bos" else (L - 1 if case == "force_eos" else 17)
    logits = (torch.randn(B * nb, V, device="cuda") * 3).to(dtype)
    beam_scores = torch.randn(B, nb, device="cuda") * 2
    # small token alphabet so earlier n-grams repeat and bans actually fire
    seqs = torch.randint(0, 12, (B * nb, L), device="cuda")
    eos = 2
    proc = (cur + 1 if case == "minlen" else None, 3 if case in ("ngram", "force_eos") else 0,
            0 if case == "force_bos" else None, eos if case == "force_eos" else None, L, eos)
    if case == "minlen":
        logits[:, eos] = 100.0  # would win every beam without the ban
    if case == "ngram":  # make a banned completion the best token of every row
        c = seqs[:, cur - 2:cur]
        seqs[:, 3:5] = c
        seqs[:, 5] = 7
        logits[:, 7] = 50.0
    cand, (ref_s, ref_i) = _composite(logits, beam_scores, seqs, cur, B, nb, proc)
    got_s, got_i = gen._beam_candidates(logits, beam_scores, seqs, cur, B, nb, proc)
    fin = torch.isfinite(ref_s)
    assert torch.equal(fin, torch.isfinite(got_s))
    # the same top scores in the same order, and every returned index names a candidate with its reported score (bf16
    # logits tie often; the kernel breaks ties by the lower index, torch.topk's order among ties is unspecified)
    torch.testing.assert_close(got_s[fin], ref_s[fin], rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(cand.gather(1, got_i)[fin], got_s[fin], rtol=1e-5, atol=1e-4)
    assert (got_i[fin] // V < nb).all()
    if case == "ngram":
        assert not (got_i % V == 7).any()


def test_generation_fused_beam_step_matches_composite(monkeypatch):
    cfg = resolve_config("bart-base").replace(num_layers=2, num_decoder_layers=2, vocab_size=4096, d_model=512,
                                              num_heads=8, d_ff=1024)
    torch.manual_seed(0)
    m = build_model(cfg).cuda().float().eval()
    ids = torch.randint(3, cfg.vocab_size, (6, 40), device="cuda")
    am = torch.ones_like(ids)
    outs = []
    for flag in ("0", "1"):
        monkeypatch.setenv("DLLM_ROUTE", f"gen_fused_beam={flag}")
        outs.append(m.generate(ids, attention_mask=am, max_length=24, num_beams=2, no_repeat_ngram_size=3,
                               min_length=5))
    assert _ext.native() is not None
    assert outs[0].shape == outs[1].shape and torch.equal(outs[0], outs[1]), (outs[0][:2], outs[1][:2])


def test_cross_attention_shared_kv_matches_per_beam_copies():
    """Beam decoding shares a batch entry's encoder K/V among its nb hypotheses (models/t5.py, models/bart.py: the
    hypotheses become query rows of one cross-attention call): == the same K/V repeated per hypothesis."""
    from distributed_llms_example_amd.ops import attention as attn_ops
    torch.manual_seed(0)
    B, nb, Sk, H, D = 5, 3, 77, 8, 64
    q = torch.randn(B * nb, 1, H, D, device="cuda").to(torch.bfloat16)
    kv = torch.randn(B, Sk, 2, H, D, device="cuda").to(torch.bfloat16)
    mask = torch.ones(B, Sk, dtype=torch.long, device="cuda")
    mask[1, -20:] = 0
    ref = attn_ops.attention_q_kv(q, kv.repeat_interleave(nb, 0), key_padding_mask=mask.repeat_interleave(nb, 0))
    got = attn_ops.attention_q_kv(q.reshape(B, nb, H, D), kv, key_padding_mask=mask)
    assert torch.equal(got.reshape(B * nb, 1, H, D), ref.reshape(B * nb, 1, H, D))


def test_generation_shared_cross_kv_runs(monkeypatch):
    cfg = resolve_config("t5-base").replace(num_layers=2, num_decoder_layers=2, vocab_size=4096, d_model=512,
                                            num_heads=8, d_kv=64, d_ff=1024)
    torch.manual_seed(0)
    m = build_model(cfg).cuda().to(torch.bfloat16).eval()
    ids = torch.randint(3, cfg.vocab_size, (5, 60), device="cuda")
    am = torch.ones_like(ids)
    am[1, -17:] = 0
    out = m.generate(ids, attention_mask=am, max_length=20, num_beams=3)
    assert out.shape[0] == 5 and out.shape[1] <= 20


@pytest.mark.parametrize("nb", [1, 2, 4])
def test_kv_reorder_in_place_matches_gather(nb):
    """csrc/beam.hip kv_reorder (in place, only changed rows, groups that kept their rows skipped) == a gather of the
    live prefix; positions past the live prefix untouched."""
    torch.manual_seed(nb)
    L2, B, T, hd, n = 6, 37, 40, 512, 23
    rows = B * nb
    cache = torch.randn(L2, rows, T, hd, device="cuda").to(torch.bfloat16)
    src = torch.arange(rows, device="cuda")
    g = torch.randint(0, nb, (B, nb), device="cuda") + torch.arange(B, device="cuda").view(B, 1) * nb
    keep = torch.rand(B, device="cuda") < 0.3  # some batch entries keep every hypothesis in place
    src = torch.where(keep.view(B, 1), src.view(B, nb), g).reshape(-1).contiguous()
    ref = cache.clone()
    ref[:, :, :n] = cache[:, :, :n].index_select(1, src)
    _ext.native().kv_reorder(cache, src, nb, n)
    assert torch.equal(cache, ref)
