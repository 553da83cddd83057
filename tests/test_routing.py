"""ops/routing.py: the one kernel-routing table — override parsing, the plan it gives for every BASELINE.json config
shape, and (GPU) that a real step launches what the plan says."""
import pytest
import torch

from distributed_llms_example_amd.ops import routing


def test_route_overrides_parse_and_fail_loudly(monkeypatch):
    monkeypatch.setenv("DLLM_ROUTE", "proj_dgrad=lib, ffn_min_rows=4096,gen_host=1")
    assert routing.get("proj_dgrad") == "lib"
    assert routing.get("ffn_min_rows") == 4096 and isinstance(routing.get("ffn_min_rows"), int)
    assert routing.get("gen_host") == 1
    assert routing.get("lmhead") == routing.DEFAULTS["lmhead"]
    s = routing.merged(lmhead="fused")
    assert "lmhead=fused" in s and "proj_dgrad=lib" in s
    monkeypatch.setenv("DLLM_ROUTE", "no_such_key=1")
    with pytest.raises(KeyError):
        routing.get("proj_fwd")
    with pytest.raises(KeyError):
        routing.merged(bogus=1)


# (config, tokens_enc, tokens_dec, d_model, d_ff, act, vocab) -> expected plan entries.  The per-GPU micro-batches are
# the bench / entry-point defaults: t5-base b=512 at 1024/128 (the headline), bart-large b=256, t5-large b=32,
# flan-t5-xl b=16, and the reference's own train-torchrun micro-batch (t5-base b=8 x GA 16).
PLANS = [
    (("t5-base b512", 512 * 1024, 512 * 128, 768, 3072, "relu", 32128),
     {"enc.proj_fwd": "hipblaslt", "enc.proj_dgrad": "w4", "dec.proj_dgrad": "w4", "enc.ffn": "w4-relu",
      "dec.ffn": "w4-relu", "lm_head": "hipblaslt+ce", "enc.wgrad": "w4-wgrad", "dec.wgrad": "w4-wgrad"}),
    (("t5-base b8", 8 * 1024, 8 * 128, 768, 3072, "relu", 32128),
     {"enc.proj_dgrad": "hipblaslt", "enc.ffn": "w4-relu", "dec.ffn": "hipblaslt+act",
      "enc.wgrad": "w4-wgrad", "dec.wgrad": "hipblaslt"}),
    (("t5-base b1 (train-accelerator)", 1024, 128, 768, 3072, "relu", 32128),
     {"enc.wgrad": "hipblaslt", "dec.wgrad": "hipblaslt", "enc.ffn": "hipblaslt+act"}),
    (("bart-large b256", 256 * 1024, 256 * 128, 1024, 4096, "gelu", 50265),
     {"enc.proj_dgrad": "w4", "dec.proj_dgrad": "w4", "enc.ffn": "pingpong-gelu", "dec.ffn": "pingpong-gelu"}),
    (("t5-large b32", 32 * 1024, 32 * 128, 1024, 4096, "relu", 32128),
     {"enc.proj_dgrad": "w4", "dec.proj_dgrad": "hipblaslt", "enc.ffn": "w4-relu", "dec.ffn": "w4-relu"}),
    (("flan-t5-xl b16", 16 * 1024, 16 * 128, 2048, 5120, "gated-gelu", 32128),
     {"enc.ffn": "hipblaslt+act", "enc.proj_dgrad": "w4", "dec.proj_dgrad": "hipblaslt"}),
]


@pytest.mark.parametrize("args,expect", PLANS, ids=[p[0][0] for p in PLANS])
def test_route_plan_for_baseline_configs(args, expect, monkeypatch):
    """Run with the table's defaults (the test session's conftest override is removed)."""
    monkeypatch.delenv("DLLM_ROUTE", raising=False)
    plan = routing.plan(*args)
    for k, v in expect.items():
        assert plan[k] == v, (k, plan[k], v)


@pytest.mark.gpu
def test_step_launches_what_the_plan_says(monkeypatch):
    """A t5-base-shaped step (2 + 2 layers, 64 x 1024 encoder tokens: over the row thresholds) under the default
    table: the projection input gradients and the ReLU FFN run on csrc/gemm_w4.hip exactly as routing.plan says, and the
    profiler sees the hand-written kernel families of the step (w4 GEMM and FFN, attention, norms, CE, AdamW)."""
    from distributed_llms_example_amd.models import build_model, resolve_config
    from distributed_llms_example_amd.ops import ffn as ffn_mod, gemm as gemm_mod
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.engine import TrainEngine
    monkeypatch.delenv("DLLM_ROUTE", raising=False)
    cfg = resolve_config("t5-base").replace(num_layers=2, num_decoder_layers=2)
    B, S, T = 64, 1024, 128
    plan = routing.plan("t5-base", B * S, B * T, cfg.d_model, cfg.d_ff, "relu", cfg.vocab_size)
    assert plan["enc.proj_dgrad"] == "w4" and plan["enc.ffn"] == "w4-relu"
    env = init_distributed()
    torch.manual_seed(0)
    eng = TrainEngine(build_model(cfg), env, lr=1e-4, dtype=torch.bfloat16)
    eng.train()
    g = torch.Generator().manual_seed(0)
    batch = {"input_ids": torch.randint(3, cfg.vocab_size, (B, S), generator=g).cuda(),
             "attention_mask": torch.ones(B, S, dtype=torch.long).cuda(),
             "labels": torch.randint(3, cfg.vocab_size, (B, T), generator=g).cuda()}
    eng.forward_backward(batch)
    eng.step()
    torch.cuda.synchronize()
    w4_0, ffn_0 = gemm_mod.w4_calls, ffn_mod.w4_ffn_calls
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        eng.forward_backward(batch)
        eng.step()
        torch.cuda.synchronize()
    # encoder (64K rows) input gradients on w4; decoder rows (8K) under the 16K-row floor
    assert gemm_mod.w4_calls - w4_0 >= cfg.num_layers, gemm_mod.w4_calls - w4_0
    # every ReLU FFN on w4: encoder (64K rows) and decoder (8K rows, ffn_w4_min_rows = 0)
    assert ffn_mod.w4_ffn_calls - ffn_0 == cfg.num_layers + cfg.num_decoder_layers
    names = " ".join(e.key for e in prof.key_averages())
    for fam in ("gemm_w4_kernel", "attn_fwd_kernel", "attn_bwd_dq_kernel", "attn_bwd_dkdv2_kernel",
                "norm_fwd_kernel", "norm_bwd_kernel", "adamw8_kernel", "splitk_reduce_kernel"):
        assert fam in names, (fam, names[:2000])
