"""Generation parity vs transformers' GenerationMixin on CPU (greedy and beam search, KV cache)."""
import pytest
import torch

from distributed_llms_example_amd.models import build_model
from hf_oracle import hf_model_for


def _pair(name):
    torch.manual_seed(0)
    ours = build_model(name).eval()
    if hasattr(ours, "lm_head"):
        with torch.no_grad():
            ours.lm_head.weight.copy_(ours.shared.weight)
    hf = hf_model_for(ours).eval()
    return ours, hf


@pytest.mark.parametrize("name", ["t5-tiny", "umt5-tiny", "bart-tiny", "mbart-tiny", "pegasus-tiny", "marian-tiny", "m2m100-tiny", "plbart-tiny", "blenderbot-tiny"])
@pytest.mark.parametrize("beams", [1, 2, 3])
def test_generate_matches_hf(name, beams):
    ours, hf = _pair(name)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(4, ours.config.vocab_size, (3, 17), generator=g)
    am = torch.ones_like(ids)
    am[2, 12:] = 0
    ids[2, 12:] = ours.config.pad_token_id
    kw = dict(max_length=12, num_beams=beams, min_length=0, no_repeat_ngram_size=0, length_penalty=1.0,
              early_stopping=False)
    a = ours.generate(ids, attention_mask=am, **kw)
    extra = {}
    if ours.config.model_type != "t5":
        extra = dict(forced_bos_token_id=ours.config.forced_bos_token_id,
                     forced_eos_token_id=ours.config.forced_eos_token_id)
    b = hf.generate(ids, attention_mask=am, do_sample=False, **kw, **extra)
    L = min(a.shape[1], b.shape[1])
    assert torch.equal(a[:, :L], b[:, :L]), (a, b)


def test_no_repeat_ngram_and_min_length():
    ours, hf = _pair("bart-tiny")
    ids = torch.randint(4, 500, (2, 9), generator=torch.Generator().manual_seed(3))
    kw = dict(max_length=14, num_beams=2, min_length=6, no_repeat_ngram_size=2, length_penalty=2.0,
              early_stopping=True)
    a = ours.generate(ids, **kw)
    b = hf.generate(ids, do_sample=False, forced_bos_token_id=0, forced_eos_token_id=2, **kw)
    L = min(a.shape[1], b.shape[1])
    assert torch.equal(a[:, :L], b[:, :L]), (a, b)


@pytest.mark.parametrize("name", ["t5-tiny", "bart-tiny"])
@pytest.mark.parametrize("beams,early,lp,ngram,minlen", [
    (2, False, 1.0, 0, 0), (3, True, 2.0, 3, 4), (4, "never", 0.5, 2, 0), (2, False, 1.0, 0, 6)])
def test_device_beam_search_matches_host_loop(name, beams, early, lp, ngram, minlen, monkeypatch):
    """Device-side beam bookkeeping == the per-step host loop (routing gen_host=1) on an eos-heavy model, so finished
    hypotheses, the stopping rule and the finalize path are all exercised."""
    torch.manual_seed(0)
    m = build_model(name).eval()
    eos = m.config.eos_token_id
    orig = m.lm_logits

    def lm_logits(h):  # a state-dependent eos boost: hypotheses finish at many different steps
        x = orig(h)
        x[..., eos] = x[..., eos] + 6.0 * torch.sin(h.float().sum(-1) * 7.0) + 1.0
        return x

    m.lm_logits = lm_logits
    g = torch.Generator().manual_seed(beams)
    ids = torch.randint(4, m.config.vocab_size, (4, 15), generator=g)
    kw = dict(max_length=16, num_beams=beams, min_length=minlen, no_repeat_ngram_size=ngram, length_penalty=lp,
              early_stopping=early)
    monkeypatch.setenv("DLLM_ROUTE", "gen_check_every=3")
    a = m.generate(ids, **kw)
    monkeypatch.setenv("DLLM_ROUTE", "gen_check_every=3,gen_host=1")
    b = m.generate(ids, **kw)
    assert torch.equal(a, b), (a, b)
    assert int((a == eos).sum()) >= 2


def test_greedy_trims_steps_after_all_done(monkeypatch):
    torch.manual_seed(0)
    m = build_model("bart-tiny").eval()
    ids = torch.randint(4, 500, (2, 9), generator=torch.Generator().manual_seed(3))
    monkeypatch.setenv("DLLM_ROUTE", "gen_check_every=1")
    a = m.generate(ids, max_length=20, num_beams=1)
    monkeypatch.setenv("DLLM_ROUTE", "gen_check_every=7")
    b = m.generate(ids, max_length=20, num_beams=1)
    assert torch.equal(a, b)
