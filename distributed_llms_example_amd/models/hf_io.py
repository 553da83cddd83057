"""HF-compatible checkpoint I/O: ``config.json`` + ``generation_config.json`` + ``model.safetensors``.

The reference saves with ``model.save_pretrained(output_dir)`` (ref/helpers.py:13); the files it
writes are reproduced here so ``transformers.AutoModelForSeq2SeqLM.
from_pretrained(our_output)`` loads our checkpoints and we load theirs.  Internally q/k/v,
cross-attention k/v and gated wi_0/wi_1 are fused weights (models/t5.py, models/bart.py); this module
splits/concatenates them.  Tied weights are stored once (``shared.weight`` /
``model.shared.weight``), as safetensors de-duplication does in ``save_pretrained``.
Loading uses safetensors only — nothing that can execute code from the file.
"""
from __future__ import annotations

import os

import torch
from safetensors.torch import load_file, save_file

from .bart import BartForConditionalGeneration
from .config import Seq2SeqConfig, resolve_config
from .t5 import T5ForConditionalGeneration

_FUSED_T5 = {".qkv.weight": [".q.weight", ".k.weight", ".v.weight"], ".kv.weight": [".k.weight", ".v.weight"]}
_FUSED_BART = {".qkv_proj.": [".q_proj.", ".k_proj.", ".v_proj."], ".kv_proj.": [".k_proj.", ".v_proj."]}


def build_model(cfg_or_name, dtype=torch.float32, device="cpu"):
    cfg = cfg_or_name if isinstance(cfg_or_name, Seq2SeqConfig) else resolve_config(cfg_or_name)
    cls = T5ForConditionalGeneration if cfg.model_type == "t5" else BartForConditionalGeneration
    with torch.device(device):
        model = cls(cfg)
    return model.to(dtype=dtype)


def to_hf_state_dict(model) -> dict[str, torch.Tensor]:
    cfg: Seq2SeqConfig = model.config
    out = {}
    for name, t in model.state_dict().items():
        t = t.detach()
        if cfg.model_type == "t5":
            if name.endswith(".wi.weight") and cfg.is_gated:
                a, b = t.chunk(2, dim=0)
                out[name.replace(".wi.weight", ".wi_0.weight")] = a
                out[name.replace(".wi.weight", ".wi_1.weight")] = b
                continue
            done = False
            for suf, parts in _FUSED_T5.items():
                if name.endswith(suf):
                    for part, piece in zip(parts, t.chunk(len(parts), dim=0)):
                        out[name[: -len(suf)] + part] = piece
                    done = True
            if not done:
                out[name] = t
        else:
            done = False
            for key, parts in _FUSED_BART.items():
                if key in name:
                    for part, piece in zip(parts, t.chunk(len(parts), dim=0)):
                        out[name.replace(key, part)] = piece
                    done = True
            if not done:
                out[name] = t
    return {k: v.contiguous() for k, v in out.items()}


def from_hf_state_dict(model, sd: dict[str, torch.Tensor], strict: bool = True):
    cfg: Seq2SeqConfig = model.config
    own = model.state_dict()
    new = {}
    for name in own:
        if cfg.model_type == "t5":
            if name.endswith(".wi.weight") and cfg.is_gated:
                new[name] = torch.cat([sd[name.replace(".wi.weight", ".wi_0.weight")],
                                       sd[name.replace(".wi.weight", ".wi_1.weight")]], 0)
                continue
            hit = None
            for suf, parts in _FUSED_T5.items():
                if name.endswith(suf):
                    hit = torch.cat([sd[name[: -len(suf)] + p] for p in parts], 0)
            if hit is not None:
                new[name] = hit
            elif name in sd:
                new[name] = sd[name]
            elif name == "lm_head.weight" and "shared.weight" in sd:
                new[name] = sd["shared.weight"]
        else:
            hit = None
            for key, parts in _FUSED_BART.items():
                if key in name:
                    hit = torch.cat([sd[name.replace(key, p)] for p in parts], 0)
            if hit is not None:
                new[name] = hit
            elif name in sd:
                new[name] = sd[name]
            elif name.endswith("shared.weight") and "model.shared.weight" not in sd and "lm_head.weight" in sd:
                new[name] = sd["lm_head.weight"]
    # fixed sinusoidal position tables are a function of (max_position_embeddings, d_model): transformers' Marian drops
    # them on save (_keys_to_ignore_on_save) and our module already holds the exact table, so their absence is not an
    # error (Pegasus checkpoints do carry them and they are loaded like any other key)
    derived = {n + ".weight" for n, m in model.named_modules() if getattr(m, "derived_table", False)}
    missing = [k for k in own if k not in new and k not in derived]
    if strict and missing:
        raise KeyError(f"missing keys in checkpoint: {missing[:8]}{'...' if len(missing) > 8 else ''}")
    with torch.no_grad():
        for k, v in new.items():
            own[k].copy_(v.to(own[k].dtype))
    return missing


def save_pretrained(model, output_dir: str, dtype=torch.float32) -> list[str]:
    """Write config.json, generation_config.json, model.safetensors.  Returns written file names."""
    os.makedirs(output_dir, exist_ok=True)
    model.config.save(output_dir)
    sd = {k: v.to("cpu", dtype=dtype if v.is_floating_point() else v.dtype) for k, v in to_hf_state_dict(model).items()}
    save_file(sd, os.path.join(output_dir, "model.safetensors"), metadata={"format": "pt"})
    return ["config.json", "generation_config.json", "model.safetensors"]


def from_pretrained(name_or_path: str, dtype=torch.float32, device="cpu"):
    """Build a model from a preset name / HF id (random init, HF init rules) or from a directory
    written by us or by ``transformers`` (``model.safetensors``)."""
    cfg = resolve_config(name_or_path)
    model = build_model(cfg, dtype=torch.float32, device="cpu")
    if name_or_path and os.path.isdir(name_or_path):
        st = os.path.join(name_or_path, "model.safetensors")
        if os.path.exists(st):
            from_hf_state_dict(model, load_file(st))
    return model.to(device=device, dtype=dtype)
