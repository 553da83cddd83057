"""Learning-rate schedules (host-side scalars, no host<->device sync).

``linear``: warmup then linear decay to 0 — transformers optimization.py:101-104 (lr_lambda of
get_linear_schedule_with_warmup), the schedule the reference uses everywhere
(``lr_scheduler_type`` default in the Trainer path; ``get_scheduler('linear', ...)`` at
ref/train-accelerator.py:200-205 and ref/train-task.py:266-271).
"""
from __future__ import annotations

import math


def lr_lambda(name: str, step: int, warmup: int, total: int) -> float:
    if name == "constant":
        return 1.0
    if name == "constant_with_warmup":
        return step / max(1, warmup) if step < warmup else 1.0
    if step < warmup:
        return float(step) / float(max(1, warmup))
    if name == "linear":
        return max(0.0, float(total - step) / float(max(1, total - warmup)))
    if name == "cosine":
        prog = float(step - warmup) / float(max(1, total - warmup))
        return max(0.0, 0.5 * (1.0 + math.cos(math.pi * prog)))
    raise ValueError(f"unknown schedule {name!r}")


class LRScheduler:
    """Mirrors torch's LambdaLR bookkeeping: ``get_last_lr()`` after ``step()``."""

    def __init__(self, optimizer, name: str = "linear", num_warmup_steps: int = 0, num_training_steps: int = 1):
        self.optimizer = optimizer
        self.name = name
        self.warmup = num_warmup_steps
        self.total = num_training_steps
        self.base_lr = optimizer.param_groups[0].get("initial_lr", optimizer.param_groups[0]["lr"])
        self.last_step = 0
        self._apply()

    def _apply(self):
        lr = self.base_lr * lr_lambda(self.name, self.last_step, self.warmup, self.total)
        for g in self.optimizer.param_groups:
            g["lr"] = lr

    def step(self):
        self.last_step += 1
        self._apply()

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        return {"name": self.name, "warmup": self.warmup, "total": self.total, "base_lr": self.base_lr,
                "last_step": self.last_step}

    def load_state_dict(self, d):
        # like torch LambdaLR: restore the step counter and base lr; the schedule shape (warmup, total)
        # comes from the resuming run's arguments
        self.base_lr, self.last_step = d["base_lr"], d["last_step"]
        self._apply()
