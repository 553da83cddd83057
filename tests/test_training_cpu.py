"""Training-loop semantics on CPU (SURVEY.md §4 level 3): schedule, optimizer, clip, checkpoint
round-trip through transformers, resume, collator, ROUGE, dropout RNG."""
import json
import math
import os

import numpy as np
import pytest
import torch

from distributed_llms_example_amd.data.collator import DataCollatorForSeq2Seq
from distributed_llms_example_amd.models import build_model, from_pretrained, save_pretrained
from distributed_llms_example_amd.ops import rng
from distributed_llms_example_amd.ops.optim import FusedAdamW
from distributed_llms_example_amd.parallel.flat import FlatParams
from distributed_llms_example_amd.train import rouge
from distributed_llms_example_amd.train.schedule import LRScheduler, lr_lambda


def test_linear_schedule_matches_transformers():
    from transformers import get_linear_schedule_with_warmup
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=5e-5)
    ref = get_linear_schedule_with_warmup(opt, 7, 40)
    fake = FusedAdamW.__new__(FusedAdamW)
    fake.param_groups = [{"lr": 5e-5, "initial_lr": 5e-5}]
    ours = LRScheduler(fake, "linear", 7, 40)
    for _ in range(45):
        assert abs(ours.get_last_lr()[0] - ref.get_last_lr()[0]) < 1e-12
        opt.step()
        ref.step()
        ours.step()
    assert lr_lambda("cosine", 5, 0, 10) == pytest.approx(0.5)


def test_fused_adamw_reference_matches_torch_with_clip():
    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.LayerNorm(16), torch.nn.Linear(16, 4))
    m2 = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.LayerNorm(16), torch.nn.Linear(16, 4))
    m2.load_state_dict(m1.state_dict())
    flat = FlatParams(m1)
    nd = lambda n: n.endswith("bias") or n.startswith("1.")  # noqa: E731
    opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1, no_decay=nd)
    ref = torch.optim.AdamW([{"params": [p for n, p in m2.named_parameters() if not nd(n)], "weight_decay": 0.1},
                             {"params": [p for n, p in m2.named_parameters() if nd(n)], "weight_decay": 0.0}], lr=1e-2)
    for _ in range(6):
        x = torch.randn(5, 8)
        opt.zero_grad()
        ref.zero_grad()
        (m1(x).pow(2).sum() * 10).backward()
        (m2(x).pow(2).sum() * 10).backward()
        n1 = opt.step(max_grad_norm=1.0)
        n2 = torch.nn.utils.clip_grad_norm_(m2.parameters(), 1.0)
        ref.step()
        assert float(n1) == pytest.approx(float(n2), rel=1e-5)
        for a, b in zip(m1.parameters(), m2.parameters()):
            torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)


def test_checkpoint_loads_in_transformers(tmp_path):
    import transformers
    for name in ("t5-tiny", "umt5-tiny", "bart-tiny", "mbart-tiny", "pegasus-tiny", "marian-tiny", "m2m100-tiny",
                 "plbart-tiny", "blenderbot-tiny"):
        m = build_model(name).eval()
        d = tmp_path / name
        save_pretrained(m, str(d))
        # eager: transformers' SDPA path for UMT5 drops the position bias (tests/hf_oracle.py)
        hf = transformers.AutoModelForSeq2SeqLM.from_pretrained(str(d), attn_implementation="eager").eval()
        ids = torch.randint(3, 500, (2, 11))
        lab = torch.randint(3, 500, (2, 6))
        a = m(input_ids=ids, labels=lab).loss
        b = hf(input_ids=ids, labels=lab).loss
        assert float(a) == pytest.approx(float(b), rel=1e-5, abs=1e-5)
        m2 = from_pretrained(str(d)).eval()
        assert float(m2(input_ids=ids, labels=lab).loss) == pytest.approx(float(a), rel=1e-6)
        meta = json.load(open(d / "config.json"))
        assert meta["model_type"] == (m.config.t5_flavor if m.config.model_type == "t5" else m.config.model_type)


def test_trainer_resume_is_exact(tmp_path):
    """Train 6 steps straight vs 3 + resume-from-checkpoint + 3: identical weights."""
    from distributed_llms_example_amd.data.dataset import SyntheticSeq2Seq
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.trainer import Trainer, TrainingArguments
    env = init_distributed(cpu=True)
    ds = SyntheticSeq2Seq(24, 12, 6, 500, seed=1)
    coll = DataCollatorForSeq2Seq(0, 0)

    def make(out, max_steps, save_steps):
        torch.manual_seed(0)
        m = build_model("t5-tiny")
        args = TrainingArguments(output_dir=str(out), max_steps=max_steps, per_device_train_batch_size=4,
                                 learning_rate=1e-3, warmup_steps=2, logging_steps=100, save_steps=save_steps,
                                 bf16=False, seed=3)
        return Trainer(m, args, train_dataset=ds, data_collator=coll, env=env)

    t1 = make(tmp_path / "a", 6, 1000)
    t1.train()
    t2 = make(tmp_path / "b", 3, 3)
    t2.train()
    t3 = make(tmp_path / "b", 6, 1000)
    t3.train(resume_from_checkpoint=str(tmp_path / "b" / "checkpoint-3"))
    assert t3.state.global_step == 6
    torch.testing.assert_close(t1.engine.flat.param_buf, t3.engine.flat.param_buf, atol=1e-6, rtol=1e-5)


def test_collator_shift_right_and_padding():
    c = DataCollatorForSeq2Seq(pad_token_id=1, decoder_start_token_id=2, pad_to_multiple_of=8)
    feats = [{"input_ids": [5, 6, 7], "attention_mask": [1, 1, 1], "labels": [9, 10]},
             {"input_ids": [5], "attention_mask": [1], "labels": [11, 12, 13]}]
    b = c(feats)
    assert b["input_ids"].shape == (2, 8) and b["input_ids"][1, 1] == 1
    assert b["labels"].tolist()[0][:3] == [9, 10, -100]
    assert b["decoder_input_ids"].tolist()[0][:3] == [2, 9, 10]
    assert b["decoder_input_ids"].tolist()[0][3] == 1  # -100 -> pad


def test_rouge_known_values():
    s = rouge.score("the cat sat on the mat", "the cat sat on the mat")
    assert all(v == pytest.approx(1.0) for v in s.values())
    s = rouge.score("the cat was found under the bed", "the cat was under the bed")
    # unigram: P = 6/7, R = 6/6 -> F = 12/13; bigram: overlaps the cat, cat was, under the, the bed = 4 -> P 4/6 R 4/5
    assert s["rouge1"] == pytest.approx(12 / 13)
    assert s["rouge2"] == pytest.approx(2 * (4 / 6) * (4 / 5) / (4 / 6 + 4 / 5))
    assert s["rougeL"] == pytest.approx(12 / 13)
    st = rouge.PorterStemmer()
    assert [st.stem(w) for w in ("caresses", "ponies", "running", "relational", "happiness")] == \
        ["caress", "poni", "run", "relat", "happi"]
    m = rouge.load("rouge")
    m.add_batch(["a b c", "x y"], ["a b c", "z"])
    r = m.compute()
    assert r["rouge1"] == pytest.approx(0.5)


def test_dropout_rng_statistics_and_reproducibility():
    k1 = rng.keep_mask(1234, 0.1, (1000, 100), "cpu")
    k2 = rng.keep_mask(1234, 0.1, (1000, 100), "cpu")
    assert torch.equal(k1, k2)
    assert abs(1 - k1.float().mean().item() - 0.1) < 0.003
    k3 = rng.keep_mask(1235, 0.1, (1000, 100), "cpu")
    assert (k1 != k3).float().mean() > 0.1
    a = rng.attention_keep_mask(5, 0.25, 2, 3, 7, 9, "cpu")
    assert a.shape == (2, 3, 7, 9) and abs(1 - a.float().mean().item() - 0.25) < 0.08


def test_calculate_metric_on_test_ds_cpu():
    from distributed_llms_example_amd.data.tokenization import WordTokenizer
    from distributed_llms_example_amd.train.evaluation import calculate_metric_on_test_ds, generate_batch_sized_chunks
    assert [list(c) for c in generate_batch_sized_chunks(list(range(7)), 3)] == [[0, 1, 2], [3, 4, 5], [6]]
    ds = {"article": ["the cat sat on the mat", "a dog ran in the park", "birds fly south"],
          "highlights": ["cat on mat", "dog in park", "birds fly"]}
    tok = WordTokenizer.build(ds["article"] + ds["highlights"], 500)
    torch.manual_seed(0)
    m = build_model("t5-tiny")
    scores = calculate_metric_on_test_ds(m, tok, ds, batch_size=2, max_source_length=16, num_beams=2, max_length=6)
    assert set(scores) >= {"rouge1", "rouge2", "rougeL", "rougeLsum"}
    assert all(0.0 <= v <= 1.0 for v in scores.values())


def test_trainer_steps_on_epoch_remainder(tmp_path):
    """len(loader) % ga != 0: the epoch's last optimizer step takes the leftover micro-batches (HF Trainer), so
    no gradient is carried into the next epoch and ceil(len / ga) steps run per epoch."""
    from distributed_llms_example_amd.data.dataset import SyntheticSeq2Seq
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.trainer import Trainer, TrainingArguments
    env = init_distributed(cpu=True)
    ds = SyntheticSeq2Seq(5, 12, 6, 500, seed=1)  # 5 micro-batches of 1, ga = 2 -> 3 steps / epoch
    torch.manual_seed(0)
    args = TrainingArguments(output_dir=str(tmp_path), num_train_epochs=2, per_device_train_batch_size=1,
                             gradient_accumulation_steps=2, learning_rate=1e-3, logging_steps=100,
                             save_steps=1000, bf16=False, seed=3)
    t = Trainer(build_model("t5-tiny"), args, train_dataset=ds, data_collator=DataCollatorForSeq2Seq(0, 0), env=env)
    t.train()
    assert t.state.global_step == 6
    assert float(t.engine.flat.grad_buf.abs().sum()) == 0.0  # nothing left accumulated


def test_trainer_coalesced_grad_accumulation_cpu(tmp_path):
    """Gradient-accumulation micro-batches run as one padded forward/backward (coalesce_grad_accum) give the same
    training trajectory as one pass per micro-batch: same samples, same global token normalisation, one step."""
    from distributed_llms_example_amd.data.dataset import SyntheticSeq2Seq
    from distributed_llms_example_amd.models import resolve_config
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.trainer import Trainer, TrainingArguments
    env = init_distributed(cpu=True)
    ds = SyntheticSeq2Seq(12, 12, 6, 500, seed=2)
    cfg = resolve_config("t5-tiny").replace(dropout_rate=0.0, attention_dropout=0.0)
    torch.manual_seed(0)
    sd = build_model(cfg).state_dict()
    out = {}
    for cap in (0, 4, 3):  # off / whole group in one pass / passes of 3 + 1 micro-batches
        m = build_model(cfg)
        m.load_state_dict(sd)
        args = TrainingArguments(output_dir=str(tmp_path / str(cap)), num_train_epochs=1, per_device_train_batch_size=1,
                                 gradient_accumulation_steps=4, learning_rate=1e-3, logging_steps=1, save_steps=1000,
                                 bf16=False, seed=3, coalesce_grad_accum=cap)
        t = Trainer(m, args, train_dataset=ds, data_collator=DataCollatorForSeq2Seq(0, 0), env=env)
        t.train()
        assert t.state.global_step == 3
        out[cap] = (torch.cat([p.detach().flatten() for p in m.parameters()]),
                    [h["loss"] for h in t.state.log_history if "loss" in h])
    for cap in (4, 3):
        torch.testing.assert_close(out[cap][0], out[0][0], atol=2e-5, rtol=1e-4)
        assert all(abs(a - b) < 1e-3 for a, b in zip(out[cap][1], out[0][1])), (out[cap][1], out[0][1])


def test_trainer_merge_pads_like_one_collated_batch():
    """Coalescing micro-batches of different padded lengths == collating all their samples as one batch."""
    from distributed_llms_example_amd.train.trainer import Trainer
    rng = torch.Generator().manual_seed(4)
    feats = [{"input_ids": torch.randint(3, 99, (int(n),), generator=rng).tolist(),
              "labels": torch.randint(3, 99, (int(t),), generator=rng).tolist()}
             for n, t in zip(torch.randint(4, 15, (6,), generator=rng), torch.randint(2, 9, (6,), generator=rng))]
    col = DataCollatorForSeq2Seq(pad_token_id=1, decoder_start_token_id=2)
    groups = [col(feats[i:i + 2]) for i in (0, 2, 4)]
    merged = Trainer._merge(groups, pad_id=1)
    whole = col(feats)
    # decoder inputs are left to the model's shift_right of the merged labels (the collator's own rule)
    assert "decoder_input_ids" not in merged and set(merged) | {"decoder_input_ids"} == set(whole)
    for k in merged:
        assert torch.equal(merged[k], whole[k]), k
    lab = merged["labels"]
    dec = torch.cat([torch.full_like(lab[:, :1], 2), lab[:, :-1]], 1).masked_fill(
        torch.cat([torch.zeros_like(lab[:, :1], dtype=torch.bool), lab[:, :-1] == -100], 1), 1)
    assert torch.equal(dec, whole["decoder_input_ids"])  # what the model's shift_right rebuilds (D10)


def test_global_token_normalisation_cpu():
    """num_items over micro-batches with different ignored-token counts == full-batch token mean (fp32, exact)."""
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.engine import TrainEngine, token_count
    env = init_distributed(cpu=True)
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(3, 500, (4, 12), generator=g)
    lab = torch.randint(3, 500, (4, 6), generator=g)
    lab[0, 1:] = -100
    lab[3, 4:] = -100
    mbs = [{"input_ids": ids[i:i + 2], "attention_mask": torch.ones(2, 12, dtype=torch.long), "labels": lab[i:i + 2]}
           for i in (0, 2)]
    torch.manual_seed(0)
    sd = build_model("t5-tiny").state_dict()

    def eng():
        m = build_model("t5-tiny")
        m.load_state_dict(sd)
        return TrainEngine(m, env, dtype=torch.float32).train(False)

    e1 = eng()
    n = sum(token_count(b["labels"]) for b in mbs)
    for i, b in enumerate(mbs):
        e1.forward_backward(b, sync=i == 1, num_items=n)
    e2 = eng()
    e2.forward_backward({"input_ids": ids, "attention_mask": torch.ones(4, 12, dtype=torch.long), "labels": lab})
    torch.testing.assert_close(e1.flat.grad_buf, e2.flat.grad_buf, atol=1e-6, rtol=1e-4)


def test_bf16_params_fp32_grad_buffer_cpu():
    """bf16 parameters with the default fp32 gradient buffer: p.grad stays None, fused ops and the autograd
    fold-in hook (relative-position bias table) both land in the fp32 buffer; matches the fp32 model closely."""
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.engine import TrainEngine
    env = init_distributed(cpu=True)
    torch.manual_seed(0)
    sd = build_model("t5-tiny").state_dict()
    g = torch.Generator().manual_seed(1)
    b = {"input_ids": torch.randint(3, 500, (2, 16), generator=g), "attention_mask": torch.ones(2, 16, dtype=torch.long),
         "labels": torch.randint(3, 500, (2, 8), generator=g)}
    m16 = build_model("t5-tiny")
    m16.load_state_dict(sd)
    e16 = TrainEngine(m16, env, dtype=torch.bfloat16).train(False)
    assert e16.flat.grad_buf.dtype == torch.float32
    e16.forward_backward(b)
    assert all(p.grad is None for p in e16.flat.params)
    m32 = build_model("t5-tiny").eval()  # plain autograd (no FlatParams: F.embedding / F.linear paths)
    m32.load_state_dict(sd)
    m32(**b).loss.backward()
    ref = dict(m32.named_parameters())
    for seg in e16.flat.segments:
        a = e16.flat.grad_buf[seg.offset:seg.offset + seg.numel]
        r = ref[seg.name].grad.flatten()
        assert float(a.abs().sum()) > 0, seg.name
        cos = torch.nn.functional.cosine_similarity(a.double(), r.double(), dim=0).item()
        assert cos > 0.98, (seg.name, cos)


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_attention_dropout_hash_statistics(p):
    """The attention keep-mask hash (two 24-bit multiplies per key pair): rate, pair / row / column independence."""
    k = rng.attention_keep_mask(77, p, 2, 4, 256, 512, "cpu").double()
    d = 1 - k
    assert abs(d.mean().item() - p) < 0.004
    both_pair = (d[..., 0::2] * d[..., 1::2]).mean().item()      # the two keys of one hash
    both_row = (d[:, :, 0::2, :] * d[:, :, 1::2, :]).mean().item()  # adjacent query rows
    both_far = (d[..., :256] * d[..., 256:]).mean().item()
    tol = 0.0015 if p < 0.3 else 0.006
    for v in (both_pair, both_row, both_far):
        assert abs(v - p * p) < tol, (both_pair, both_row, both_far)
    # lag-2 (odd-odd, even-even: successive hashes of one row), lag-3 and lag-16 keys: independent draws give p^2
    dd = d.reshape(-1, d.shape[-1])
    oo = (dd[:, 1::2][:, :-1] * dd[:, 1::2][:, 1:]).mean().item()
    ee = (dd[:, 0::2][:, :-1] * dd[:, 0::2][:, 1:]).mean().item()
    l3 = (dd[:, :-3] * dd[:, 3:]).mean().item()
    l16 = (dd[:, :-16] * dd[:, 16:]).mean().item()
    for v in (oo, ee, l3, l16):
        assert abs(v - p * p) < tol, (oo, ee, l3, l16)
    # per-row drop counts: binomial variance Sk p (1 - p) (a hash linear in the key index had ~1/8 of it)
    var = dd.sum(1).var().item()
    binom = dd.shape[1] * p * (1 - p)
    assert 0.75 * binom < var < 1.3 * binom, (var, binom)
    # per-key-column and per-row drop rates stay near p (no stuck columns / rows)
    col = d.mean(dim=(0, 1, 2))
    row = d.mean(dim=(0, 1, 3))
    assert (col - p).abs().max().item() < 0.06 and (row - p).abs().max().item() < 0.06


def test_ffn_dropout_is_the_row_weyl_hash():
    """The FFN activations draw the row-Weyl decisions (ops/activations.py ffn_keep_mask, csrc/common.h rw_*): one
    row per token of the flattened [..., d_ff] activation, the same function as the attention mask with B = H = 1;
    drop rate p and independent adjacent rows / column pairs at the FFN shapes."""
    from distributed_llms_example_amd.ops import activations
    for act, gated in (("relu", False), ("gelu", False), ("gelu_new", True)):
        k = activations.ffn_keep_mask(act, gated, 91, 0.1, (4, 128, 768), "cpu")
        assert k.shape == (4, 128, 768)
        assert torch.equal(k.view(512, 768), rng.rowwise_keep_mask(91, 0.1, 512, 768, "cpu"))
        assert torch.equal(k.view(512, 768), rng.attention_keep_mask(91, 0.1, 1, 1, 512, 768, "cpu")[0, 0])
    d = 1 - rng.rowwise_keep_mask(5, 0.1, 2048, 3072, "cpu").double()
    assert abs(d.mean().item() - 0.1) < 0.002
    for v in ((d[0::2] * d[1::2]).mean().item(), (d[:, 0::2] * d[:, 1::2]).mean().item()):
        assert abs(v - 0.01) < 0.001, v


def test_relayout_keeps_stacked_groups_adjacent():
    """FlatParams.relayout with an order that splits a stacked group (the decoder's cross-attention K/V weights,
    consumed as ONE tensor by ops/linear.py stacked_linear): the group is re-joined at its first member's position,
    parameter values survive, and stacked_linear still finds the adjacent view."""
    import random
    from distributed_llms_example_amd.ops.linear import _adjacent
    from distributed_llms_example_amd.parallel.flat import FlatParams
    m = build_model("t5-tiny")
    flat = FlatParams(m)
    assert flat.groups, "t5 declares stacked cross-attention K/V groups"
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    order = list(range(len(flat.segments)))
    random.Random(0).shuffle(order)
    flat.relayout(order)
    for n, p in m.named_parameters():
        assert torch.equal(p.detach(), before[n]), n
    for grp in m._dllm_param_groups():
        assert _adjacent([p for p in grp]) is not None


def test_native_build_provenance_detects_stale_sources(tmp_path, monkeypatch):
    """tools/build_native.py records the sha256 of every native source in _C.build.json; the loader compares them with
    the tree and refuses a library built from other sources (distributed_llms_example_amd/_ext.py stale_sources)."""
    import json
    import shutil
    from distributed_llms_example_amd import _ext
    pkg, csrc = tmp_path / "pkg", tmp_path / "csrc"
    pkg.mkdir()
    shutil.copytree(_ext._CSRC, csrc)
    sys_path = __import__("sys").path
    sys_path.insert(0, str(__import__("pathlib").Path(_ext._CSRC).parent / "tools"))
    try:
        import build_native
    finally:
        sys_path.pop(0)
    monkeypatch.setattr(build_native, "CSRC", str(csrc))
    (pkg / "_C.build.json").write_text(json.dumps({"sources": build_native.source_hashes()}))
    monkeypatch.setattr(_ext, "_PKG", str(pkg))
    monkeypatch.setattr(_ext, "_CSRC", str(csrc))
    assert _ext.stale_sources() == []
    (csrc / "norm.hip").write_text((csrc / "norm.hip").read_text() + "\n// edited\n")
    assert _ext.stale_sources() == ["norm.hip"]


def test_step_runner_schedule_matches_eager_steps(monkeypatch):
    """train/graph.py StepRunner (what every entry point runs): eager warmup per batch shape, then capture + replays,
    eager steps for other shapes — run here with the graph's eager schedule (GraphedStep use_graph=False), it must
    give exactly the parameters of plain eager steps with the same dropout stream, and count replays correctly."""
    import functools
    from distributed_llms_example_amd.models import build_model
    from distributed_llms_example_amd.ops.rng import manual_seed
    from distributed_llms_example_amd.parallel.env import DistEnv
    from distributed_llms_example_amd.train import graph as G
    from distributed_llms_example_amd.train.engine import TrainEngine

    env = DistEnv()
    g = torch.Generator().manual_seed(1)

    def batch(B, S=12, T=6):
        return {"input_ids": torch.randint(3, 500, (B, S), generator=g),
                "attention_mask": torch.ones(B, S, dtype=torch.long), "labels": torch.randint(3, 500, (B, T), generator=g)}

    data = [batch(2) for _ in range(6)] + [batch(1)] + [batch(2)]  # a ragged batch between full ones

    def engine():
        torch.manual_seed(0)
        manual_seed(5)
        e = TrainEngine(build_model("t5-tiny"), env, lr=1e-3, dtype=torch.float32)
        e.train()
        return e

    monkeypatch.setattr(G, "GraphedStep", functools.partial(G.GraphedStep, use_graph=False))
    eng_r = engine()
    runner = G.StepRunner(eng_r, enabled=True, warmup=2)
    lr = [1e-3, 9e-4, 8e-4, 7e-4, 6e-4, 5e-4, 4e-4, 3e-4]
    lr_run = [float(runner([b], lr=l)[0][0]) for b, l in zip(data, lr)]
    assert runner.graph is not None and runner.graph_error is None
    # shapes [2]: eager x2 (warmup), capture + replay, replays ...; the batch of 1 runs eagerly
    assert runner.replays == 5 and runner.eager_steps == 3, (runner.replays, runner.eager_steps)
    p_run = eng_r.flat.param_buf.clone()
    eng_r.disable_step_seeds()

    eng_e = engine()
    eng_e.enable_step_seeds()
    le = []
    for b, l in zip(data, lr):
        le.append(float(eng_e.forward_backward(b)))
        eng_e.step(lr=l)
    eng_e.disable_step_seeds()
    assert lr_run == pytest.approx(le, rel=1e-6, abs=1e-7)
    assert torch.allclose(p_run, eng_e.flat.param_buf, rtol=1e-5, atol=1e-7)


def test_accelerator_train_step_clip_applies_to_the_next_step_only():
    """make_train_step keeps the eager meaning of clip_grad_norm_: a clip requested before a step applies
    to that step only, exactly like the explicit loop backward + PreparedOptimizer.step."""
    from distributed_llms_example_amd.models import build_model
    from distributed_llms_example_amd.train.accelerator import Accelerator

    g = torch.Generator().manual_seed(3)
    batches = [{"input_ids": torch.randint(3, 500, (2, 12), generator=g), "attention_mask": torch.ones(2, 12, dtype=torch.long),
                "labels": torch.randint(3, 500, (2, 6), generator=g)} for _ in range(3)]
    clips = [0.01, None, 0.02]

    def run(fused_step: bool):
        acc = Accelerator(cpu=True)
        torch.manual_seed(0)
        model = build_model("t5-tiny")
        opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.0)
        model, opt = acc.prepare(model, opt)
        model.train(False)
        step = acc.make_train_step(model, opt) if fused_step else None
        for b, c in zip(batches, clips):
            if c is not None:
                acc.clip_grad_norm_(model.parameters(), c)
            if fused_step:
                step(b)
            else:
                acc.backward(model(**b).loss)
                opt.step()
                opt.zero_grad()
        return torch.cat([p.detach().reshape(-1).float() for p in model.parameters()])

    a, b = run(True), run(False)
    torch.testing.assert_close(a, b, rtol=0, atol=0)


@pytest.mark.parametrize("model", ["t5-tiny", "bart-tiny"])
def test_deferred_weight_gradients_match_per_micro_batch(model, monkeypatch):
    """Gradient accumulation with the weight gradients deferred to the window's last micro-batch (ops/gemm.py
    WgradDefer: one GEMM over the concatenated tokens) == one GEMM per micro-batch; the deferral really ran; the last
    window (here shorter than grad_accum) is flushed by step()."""
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.engine import TrainEngine
    env = init_distributed(cpu=True)
    g = torch.Generator().manual_seed(1)
    mbs = [{"input_ids": torch.randint(3, 500, (2, 12), generator=g), "attention_mask": torch.ones(2, 12, dtype=torch.long),
            "labels": torch.randint(3, 500, (2, 6), generator=g)} for _ in range(4)]
    torch.manual_seed(0)
    sd = build_model(model).state_dict()
    res = []
    for mode in ("1", "0"):
        monkeypatch.setenv("DLLM_DEFER_WGRAD", mode)
        m = build_model(model)
        m.load_state_dict(sd)
        e = TrainEngine(m, env, dtype=torch.float32).train(False)
        for i, b in enumerate(mbs):
            e.forward_backward(b, grad_accum=4, sync=i == 3)
        res.append((e.flat.grad_buf.clone(), e.wgrad_defer.deferred, e.wgrad_defer.merged))
        # an open window: two micro-batches of a grad_accum=4 window, then the optimizer step flushes them
        for b in mbs[:2]:
            e.forward_backward(b, grad_accum=4, sync=False)
        assert (len(e.wgrad_defer.segs) > 0) == (mode == "1")
        e.step()
        assert not e.wgrad_defer.segs
    (g1, d1, m1), (g0, d0, m0) = res
    assert d1 > 0 and m1 > 0 and d0 == 0 and m0 == 0, (d1, m1, d0, m0)
    torch.testing.assert_close(g1, g0, atol=1e-6, rtol=1e-4)


def test_step_watchdog_reports_a_stalled_step():
    """utils/watchdog.py: a step not finished within the bound is reported with the rank, the step and the caller's
    description, and ends the process (exit function called with EXIT_STALL); finished steps never fire it."""
    import time
    from distributed_llms_example_amd.utils.watchdog import EXIT_STALL, StepWatchdog
    codes = []
    wd = StepWatchdog(rank=3, timeout_s=0.3, poll_s=0.05, describe=lambda: {"buckets_launched": 2},
                      exit_fn=codes.append)
    for s in range(3):  # fast steps
        wd.begin(s)
        wd.end()
    time.sleep(0.5)
    assert codes == [] and wd.fired is None
    wd.begin(7)  # never ends
    t0 = time.monotonic()
    while not codes and time.monotonic() - t0 < 5:
        time.sleep(0.05)
    wd.close()
    assert codes == [EXIT_STALL]
    assert "rank 3" in wd.fired and "step 7" in wd.fired and "buckets_launched" in wd.fired
    off = StepWatchdog(rank=0, timeout_s=0)
    assert not off.enabled
