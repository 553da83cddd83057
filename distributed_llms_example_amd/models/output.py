"""Model output container (the fields of transformers' Seq2SeqLMOutput the runtime uses)."""
from __future__ import annotations

from dataclasses import dataclass

import torch


@dataclass
class Seq2SeqLMOutput:
    loss: torch.Tensor | None = None
    logits: torch.Tensor | None = None
    encoder_last_hidden_state: torch.Tensor | None = None

    def __getitem__(self, i):
        return (self.loss, self.logits)[i]
