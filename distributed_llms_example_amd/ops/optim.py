"""Fused AdamW + global-norm gradient clipping over the flat parameter space.

Semantics = ``torch.optim.AdamW`` (decoupled weight decay, bias-corrected moments; the Trainer
builds it with ``fused=True``, transformers trainer_optimizer.py:202-207, the custom loops with the
foreach default, ref/train-accelerator.py:187) preceded by ``clip_grad_norm_(max_norm)``
(transformers trainer.py:2535-2539): ``coef = min(1, max_norm / (||g|| + 1e-6))``.

MI355X design: parameters live in bf16 (what the GEMMs read), the optimizer keeps fp32 master
weights + fp32 moments, all as flat buffers (parallel/flat.py).  One reduction kernel computes
||g||² into a device scalar, and ONE elementwise kernel (csrc/adamw.hip) reads that scalar, so the
step never synchronises with the host (no ``.item()``).  The grad-norm is returned as a device
tensor for logging.
"""
from __future__ import annotations

import math

import torch

from .. import _ext
from ..parallel.flat import FlatParams


class FusedAdamW:
    def __init__(self, flat: FlatParams, lr: float = 5e-5, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, no_decay=None, master_weights: bool | None = None):
        self.flat = flat
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.step_count = 0
        if master_weights is None:
            master_weights = flat.dtype != torch.float32
        self.master = flat.param_buf.float().clone() if master_weights else None
        self.exp_avg = torch.zeros(flat.numel, dtype=torch.float32, device=flat.device)
        self.exp_avg_sq = torch.zeros(flat.numel, dtype=torch.float32, device=flat.device)
        self.wd_mask = flat.decay_mask(no_decay) if (no_decay is not None and weight_decay != 0.0) else None
        if no_decay is not None and weight_decay != 0.0 and self.wd_mask is None:
            # uniform: either all decay or none
            if all(no_decay(s.name) for s in flat.segments):
                self.weight_decay = 0.0
        for attr in ("master", "exp_avg", "exp_avg_sq", "wd_mask"):
            flat.register_companion(self, attr)  # kept in step with a reducer-driven relayout (parallel/flat.py)
        self._one = torch.ones((), dtype=torch.float32, device=flat.device)
        # param_groups-like view for schedulers / logging parity with torch optimizers
        self.param_groups = [{"lr": lr, "initial_lr": lr, "weight_decay": weight_decay, "betas": betas, "eps": eps}]

    # ------------------------------------------------------------------------------------------
    def grad_norm(self) -> torch.Tensor:
        g = self.flat.grad_buf
        if _ext.use_native(g):
            return _ext.native().sq_norm(g).sqrt()
        return torch.linalg.vector_norm(g.float())

    def device_hyper(self, t: torch.Tensor, lr) -> torch.Tensor:
        """[lr, lr / bc1, 1 / sqrt(bc2)] as a device tensor from a device step count ``t`` (float, already incremented)
        and ``lr`` (float or device scalar): the AdamW kernel reads it instead of host floats, so a captured graph
        replays with the right bias corrections and learning rate every step."""
        b1, b2 = self.betas
        lr_t = lr if torch.is_tensor(lr) else torch.full_like(t, float(lr))
        bc1 = 1.0 - torch.pow(torch.full_like(t, b1), t)
        bc2 = 1.0 - torch.pow(torch.full_like(t, b2), t)
        return torch.stack([lr_t, lr_t / bc1, torch.rsqrt(bc2)]).reshape(3).float().contiguous()

    @torch.no_grad()
    def step(self, max_grad_norm: float | None = None, hyper: torch.Tensor | None = None) -> torch.Tensor | None:
        """One clip + AdamW update.  ``hyper`` (device_hyper) replaces the host lr / bias corrections (graph mode)."""
        lr = self.param_groups[0]["lr"]
        self.step_count += 1
        norm = None
        coef = self._one
        if max_grad_norm is not None and max_grad_norm > 0:
            norm = self.grad_norm()
            coef = torch.clamp(max_grad_norm / (norm + 1e-6), max=1.0)
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        p = self.flat.param_buf
        g = self.flat.grad_buf
        if _ext.use_native(p):
            _ext.native().adamw_step(p, self.master, g, self.exp_avg, self.exp_avg_sq, self.wd_mask, coef, float(lr),
                                     float(b1), float(b2), float(self.eps), float(self.weight_decay), float(bc1),
                                     float(bc2), hyper)
        else:
            if hyper is not None:
                lr, bc1, bc2 = float(hyper[0]), float(hyper[0] / hyper[1]), float(1.0 / hyper[2] ** 2)
            self._reference_step(p, g, coef, lr, b1, b2, bc1, bc2)
        return norm

    def _reference_step(self, p, g, coef, lr, b1, b2, bc1, bc2):
        master = self.master if self.master is not None else p
        gf = g.float() * coef
        if self.weight_decay != 0.0:
            if self.wd_mask is None:
                master.mul_(1.0 - lr * self.weight_decay)
            else:
                master.sub_(master * self.wd_mask.float() * (lr * self.weight_decay))
        self.exp_avg.lerp_(gf, 1.0 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(gf, gf, value=1.0 - b2)
        denom = (self.exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(self.eps)
        master.addcdiv_(self.exp_avg, denom, value=-lr / bc1)
        if self.master is not None:
            p.copy_(master)

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.flat.zero_grad()

    # ------------------------------------------------------------------------------------------
    def state_dict(self) -> dict:
        """Flat state in the model's canonical (construction) segment order, whatever the current layout."""
        f = self.flat
        can = f.to_canonical
        return {"step": self.step_count, "exp_avg": can(self.exp_avg), "exp_avg_sq": can(self.exp_avg_sq),
                "master": can(self.master) if self.master is not None else None, "lr": self.param_groups[0]["lr"],
                "betas": list(self.betas), "eps": self.eps, "weight_decay": self.weight_decay,
                "layout": [{"name": n, "numel": s.numel} for n, s in
                           zip(f.canonical, sorted(f.segments, key=lambda s: f.canonical.index(s.name)))]}

    def load_state_dict(self, d: dict) -> None:
        f = self.flat
        by_name = {s.name: s.numel for s in f.segments}
        if [s["numel"] for s in d["layout"]] != [by_name.get(n) for n in f.canonical]:
            raise ValueError("optimizer state layout does not match the model")
        self.step_count = int(d["step"])
        self.exp_avg.copy_(f.from_canonical(d["exp_avg"].to(self.exp_avg.device)))
        self.exp_avg_sq.copy_(f.from_canonical(d["exp_avg_sq"].to(self.exp_avg_sq.device)))
        if self.master is not None and d.get("master") is not None:
            self.master.copy_(f.from_canonical(d["master"].to(self.master.device)))
            self.flat.param_buf.copy_(self.master)
        self.param_groups[0]["lr"] = d.get("lr", self.param_groups[0]["lr"])
