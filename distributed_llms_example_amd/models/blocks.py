"""Per-block execution policy shared by the T5 and BART stacks.

Every block runs under its own dropout seed stream (ops/rng.py ``rng_scope``) drawn from the outer stream,
so with activation checkpointing (``Seq2SeqConfig.gradient_checkpointing``; SURVEY.md §5.7 item 2, for the
flan-t5-xl long-sequence config) the block can be recomputed in backward with bit-identical dropout masks.
Recomputation uses torch's non-reentrant checkpoint: the fused ops' saved tensors are dropped after the
forward and rebuilt on first use in backward; gradient-accumulation fusion and the reducer hooks behave
exactly as without checkpointing.
"""
from __future__ import annotations

import torch
from torch.utils.checkpoint import checkpoint as _checkpoint

from ..ops.rng import default_rng, rng_scope


def run_block(fn, *args, checkpoint: bool = False):
    seed = default_rng().next_seed()

    def scoped(*a):
        with rng_scope(seed):
            return fn(*a)

    if checkpoint and torch.is_grad_enabled():
        return _checkpoint(scoped, *args, use_reentrant=False, preserve_rng_state=False)
    return scoped(*args)
