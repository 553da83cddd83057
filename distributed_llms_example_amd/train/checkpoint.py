"""Checkpoint / resume.

Model weights are written HF-compatibly (models/hf_io.py: config.json, generation_config.json,
model.safetensors).  Training state for resume — flat fp32 master weights, Adam moments, step,
scheduler, dropout-RNG / torch RNG states per rank, sampler epoch/position, TrainerState — goes to
``training_state.pt`` (tensors only, loadable with ``weights_only=True``) plus ``trainer_state.json``.
Only rank 0 writes shared files; every rank writes its own ``rng_state_<rank>.pt``; a barrier
follows (fixes the every-rank-writes race of ref/helpers.py, Appendix A Q8).
"""
from __future__ import annotations

import json
import os
import re

import torch

from ..models.hf_io import from_hf_state_dict, save_pretrained
from ..ops import rng as _rng_mod
from ..ops.rng import default_rng
from ..parallel import collectives


def save_checkpoint(path: str, model, optimizer=None, scheduler=None, trainer_state=None, extra: dict | None = None,
                    rank: int = 0, device=None):
    os.makedirs(path, exist_ok=True)
    if rank == 0:
        save_pretrained(model, path)
        state = {}
        if optimizer is not None:
            od = optimizer.state_dict()
            state["optimizer"] = {k: v for k, v in od.items() if k != "layout"}
            state["optimizer_layout"] = json.dumps(od.get("layout", []))
        if scheduler is not None:
            state["scheduler"] = scheduler.state_dict()
        if extra:
            state["extra"] = extra
        torch.save(state, os.path.join(path, "training_state.pt"))
        if trainer_state is not None:
            trainer_state.save_to_json(os.path.join(path, "trainer_state.json"))
    rng = {"dropout": default_rng().state_dict(), "torch": torch.get_rng_state()}
    st = _rng_mod._active_step[0]
    if st is not None and st.enabled:  # graph-replayable dropout (ops/rng.py StepSeed): the device step counter
        rng["step_seed"] = int(st.host)
    if torch.cuda.is_available():
        rng["cuda"] = torch.cuda.get_rng_state()
    torch.save(rng, os.path.join(path, f"rng_state_{rank}.pt"))
    collectives.barrier(device=device)


def load_checkpoint(path: str, model=None, optimizer=None, scheduler=None, rank: int = 0) -> dict:
    out = {}
    if model is not None:
        from safetensors.torch import load_file
        from_hf_state_dict(model, load_file(os.path.join(path, "model.safetensors")))
    sp = os.path.join(path, "training_state.pt")
    if os.path.exists(sp):
        state = torch.load(sp, map_location="cpu", weights_only=True)
        if optimizer is not None and "optimizer" in state:
            od = dict(state["optimizer"])
            od["layout"] = json.loads(state.get("optimizer_layout", "[]"))
            optimizer.load_state_dict(od)
        if scheduler is not None and "scheduler" in state:
            scheduler.load_state_dict(state["scheduler"])
        out["extra"] = state.get("extra", {})
    rp = os.path.join(path, f"rng_state_{rank}.pt")
    if os.path.exists(rp):
        rng = torch.load(rp, map_location="cpu", weights_only=True)
        default_rng().load_state_dict(rng["dropout"])
        if "step_seed" in rng:
            out["step_seed"] = int(rng["step_seed"])
        torch.set_rng_state(rng["torch"])
        if "cuda" in rng and torch.cuda.is_available():
            torch.cuda.set_rng_state(rng["cuda"])
    tp = os.path.join(path, "trainer_state.json")
    if os.path.exists(tp):
        with open(tp) as f:
            out["trainer_state"] = json.load(f)
    return out


def latest_checkpoint(output_dir: str) -> str | None:
    if not os.path.isdir(output_dir):
        return None
    cks = [d for d in os.listdir(output_dir) if re.fullmatch(r"checkpoint-\d+", d)]
    if not cks:
        return None
    return os.path.join(output_dir, max(cks, key=lambda d: int(d.split("-")[1])))
