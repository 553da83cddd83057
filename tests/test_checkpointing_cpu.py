"""Activation checkpointing: recomputed blocks reproduce the dropout masks exactly, so the
loss and every gradient match the non-checkpointed run bit-for-bit on the reference path."""
import copy

import pytest
import torch

from distributed_llms_example_amd.models import build_model
from distributed_llms_example_amd.ops.rng import manual_seed


@pytest.mark.parametrize("name", ["t5-tiny", "t5-tiny-gated", "bart-tiny"])
def test_checkpointing_matches_plain(name):
    torch.manual_seed(0)
    m = build_model(name)
    if name == "bart-tiny":  # exercise attention/activation dropout too
        m.config.attention_dropout = 0.1
        m.config.activation_dropout = 0.1
    m.train()
    mc = copy.deepcopy(m)
    mc.gradient_checkpointing_enable()
    assert mc.config.gradient_checkpointing and not m.config.gradient_checkpointing
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(3, 500, (3, 17), generator=g)
    am = torch.ones_like(ids)
    am[1, -4:] = 0
    lab = torch.randint(3, 500, (3, 7), generator=g)
    outs = []
    for model in (m, mc):
        manual_seed(11)
        out = model(input_ids=ids, attention_mask=am, labels=lab)
        out.loss.backward()
        outs.append(out.loss.detach())
    torch.testing.assert_close(outs[0], outs[1], rtol=0, atol=0)
    for (n, a), (_, b) in zip(m.named_parameters(), mc.named_parameters()):
        if a.grad is None:
            assert b.grad is None, n
            continue
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-7, msg=n)
