"""Trainer callback system (transformers trainer_callback.py semantics, the subset the reference uses).

``PrinterCallback`` reproduces ref/train-torchrun.py:144-147: pop ``total_flos`` and print every log
dict as one JSON line (Valohai metadata).  ``DefaultFlowCallback`` decides log / eval / save steps
(trainer_callback.py:563-621), including the final-step eval/save of transformers 5.15.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field


@dataclass
class TrainerState:
    epoch: float = 0.0
    global_step: int = 0
    max_steps: int = 0
    num_train_epochs: int = 0
    log_history: list = field(default_factory=list)
    best_metric: float | None = None
    total_flos: float = 0.0
    is_world_process_zero: bool = True
    # coalesced gradient accumulation: the per-pass budget chosen (0 = off) and its unit; a resumed run reuses it.
    # "padded_tokens" (samples x padded source + target length, Trainer._padded_tokens); checkpoints written before the
    # unit was recorded hold a budget in samples (unit None)
    coalesce_cap: int | None = None
    coalesce_cap_unit: str | None = None

    def save_to_json(self, path):
        with open(path, "w") as f:
            json.dump(dataclasses.asdict(self), f, indent=2, sort_keys=True)

    @classmethod
    def load_from_json(cls, path):
        with open(path) as f:
            d = json.load(f)
        known = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in known})


@dataclass
class TrainerControl:
    should_log: bool = False
    should_evaluate: bool = False
    should_save: bool = False
    should_training_stop: bool = False

    def reset_step(self):
        self.should_log = self.should_evaluate = self.should_save = False


class TrainerCallback:
    def on_train_begin(self, args, state, control, **kw): pass
    def on_train_end(self, args, state, control, **kw): pass
    def on_epoch_begin(self, args, state, control, **kw): pass
    def on_epoch_end(self, args, state, control, **kw): pass
    def on_step_end(self, args, state, control, **kw): pass
    def on_log(self, args, state, control, logs=None, **kw): pass
    def on_evaluate(self, args, state, control, metrics=None, **kw): pass
    def on_save(self, args, state, control, **kw): pass


class DefaultFlowCallback(TrainerCallback):
    def on_step_end(self, args, state, control, **kw):
        s = state.global_step
        if args.logging_steps > 0 and s % args.logging_steps == 0:
            control.should_log = True
        if args.eval_strategy == "steps" and args.eval_steps and s % args.eval_steps == 0:
            control.should_evaluate = True
        if args.save_strategy == "steps" and args.save_steps and s % int(args.save_steps) == 0:
            control.should_save = True
        if s >= state.max_steps:
            control.should_training_stop = True
            if args.eval_strategy == "steps":
                control.should_evaluate = True
            if args.save_strategy == "steps":
                control.should_save = True

    def on_epoch_end(self, args, state, control, **kw):
        if args.eval_strategy == "epoch":
            control.should_evaluate = True
        if args.save_strategy == "epoch":
            control.should_save = True


class PrinterCallback(TrainerCallback):
    """ref/train-torchrun.py:144-147."""

    def on_log(self, args, state, control, logs=None, **kw):
        if not state.is_world_process_zero or logs is None:
            return
        logs = dict(logs)
        logs.pop("total_flos", None)
        print(json.dumps(logs), flush=True)


class CallbackHandler:
    def __init__(self, callbacks):
        self.callbacks = []
        for c in callbacks:
            self.callbacks.append(c() if isinstance(c, type) else c)

    def add(self, cb):
        self.callbacks.append(cb() if isinstance(cb, type) else cb)

    def fire(self, event, args, state, control, **kw):
        for c in self.callbacks:
            getattr(c, event)(args, state, control, **kw)
        return control
