"""Comparator: the reference's runtime stack (HF transformers T5 + torch AdamW) on one GPU.

BASELINE.md publishes no numbers, so the number to beat is the reference stack itself
(HF `T5ForConditionalGeneration` + `torch.optim.AdamW`, as driven by
ref/train-accelerator.py:219-225 / HF Trainer) measured on MI355X with synthetic
data and random-init weights, same shapes as bench.py.

Usage: python tools/hf_comparator.py --model t5-base --batch 16 --src 1024 --tgt 128 --prec bf16-amp
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t5_config(name):
    from transformers import T5Config
    cfgs = {
        "t5-small": dict(d_model=512, d_kv=64, d_ff=2048, num_layers=6, num_heads=8),
        "t5-base": dict(d_model=768, d_kv=64, d_ff=3072, num_layers=12, num_heads=12),
        "t5-large": dict(d_model=1024, d_kv=64, d_ff=4096, num_layers=24, num_heads=16),
    }
    return T5Config(vocab_size=32128, pad_token_id=0, eos_token_id=1, decoder_start_token_id=0, **cfgs[name])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="t5-base")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--src", type=int, default=1024)
    ap.add_argument("--tgt", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--prec", default="bf16-amp", choices=["fp32", "bf16-amp", "bf16"])
    ap.add_argument("--attn", default="sdpa")
    a = ap.parse_args()
    import transformers
    from distributed_llms_example_amd.models.config import resolve_config
    torch.manual_seed(0)
    ours = resolve_config(a.model)  # same architecture presets as bench.py (config.json-compatible dict)
    d = ours.to_hf_dict()
    if ours.model_type == "t5":
        cfg = transformers.T5Config(**{k: v for k, v in d.items() if k not in ("architectures", "model_type")})
        cls = transformers.T5ForConditionalGeneration
    else:
        cfg = transformers.BartConfig(**{k: v for k, v in d.items() if k not in ("architectures", "model_type")})
        cls = transformers.BartForConditionalGeneration
    cfg._attn_implementation = a.attn
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    model = cls(cfg).to(dev)
    if a.prec == "bf16":
        model = model.to(torch.bfloat16)
    model.train()
    opt = torch.optim.AdamW(model.parameters(), lr=5e-5, fused=torch.cuda.is_available())
    V = cfg.vocab_size
    ids = torch.randint(2, V, (a.batch, a.src), device=dev)
    am = torch.ones_like(ids)
    labels = torch.randint(2, V, (a.batch, a.tgt), device=dev)

    def step():
        with torch.autocast(dev, dtype=torch.bfloat16, enabled=(a.prec == "bf16-amp")):
            out = model(input_ids=ids, attention_mask=am, labels=labels)
        out.loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return out.loss

    for _ in range(a.warmup):
        step()
    torch.cuda.is_available() and torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.is_available() and torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"stack": "hf-transformers", "model": a.model, "prec": a.prec, "attn": a.attn,
                      "batch": a.batch, "src": a.src, "tgt": a.tgt, "ms_per_step": dt * 1e3,
                      "samples_per_s": a.batch / dt, "loss": float(loss),
                      "max_mem_gb": (torch.cuda.max_memory_allocated() / 2**30 if torch.cuda.is_available() else 0)}), flush=True)


if __name__ == "__main__":
    main()
