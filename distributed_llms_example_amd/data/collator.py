"""Seq2seq batch collation (transformers DataCollatorForSeq2Seq semantics, data_collator.py:487-615).

* inputs padded to the batch max (or ``pad_to_multiple_of``) with ``pad_token_id``, mask with 0;
* labels padded with ``label_pad_token_id`` (-100);
* ``decoder_input_ids = model.prepare_decoder_input_ids_from_labels(labels)`` (shift right with the
  decoder start token, -100 → pad; modeling_t5.py:618-637, modeling_bart.py:58-71).

Returns int64 CPU tensors; ``pin_memory`` lets the device copy run async (non_blocking).
"""
from __future__ import annotations

import numpy as np
import torch


class DataCollatorForSeq2Seq:
    def __init__(self, pad_token_id: int = 0, decoder_start_token_id: int = 0, pad_to_multiple_of: int | None = None,
                 label_pad_token_id: int = -100, with_decoder_inputs: bool = True, pin_memory: bool = False):
        self.pad_token_id = pad_token_id
        self.decoder_start_token_id = decoder_start_token_id
        self.pad_to_multiple_of = pad_to_multiple_of
        self.label_pad_token_id = label_pad_token_id
        self.with_decoder_inputs = with_decoder_inputs
        self.pin_memory = pin_memory

    @classmethod
    def for_model(cls, model_or_cfg, **kw):
        cfg = getattr(model_or_cfg, "config", model_or_cfg)
        return cls(pad_token_id=cfg.pad_token_id, decoder_start_token_id=cfg.decoder_start_token_id, **kw)

    def _target(self, n):
        m = self.pad_to_multiple_of
        return n if not m else (n + m - 1) // m * m

    def _pad(self, seqs, value):
        L = self._target(max(len(s) for s in seqs))
        out = np.full((len(seqs), L), value, dtype=np.int64)
        for i, s in enumerate(seqs):
            out[i, : len(s)] = s
        return torch.from_numpy(out)

    def __call__(self, features):
        ids = self._pad([np.asarray(f["input_ids"]) for f in features], self.pad_token_id)
        if "attention_mask" in features[0]:
            am = self._pad([np.asarray(f["attention_mask"]) for f in features], 0)
        else:
            am = (ids != self.pad_token_id).long()
        batch = {"input_ids": ids, "attention_mask": am}
        if "labels" in features[0]:
            labels = self._pad([np.asarray(f["labels"]) for f in features], self.label_pad_token_id)
            batch["labels"] = labels
            if self.with_decoder_inputs:
                dec = torch.full_like(labels, self.pad_token_id)
                dec[:, 1:] = labels[:, :-1]
                dec[:, 0] = self.decoder_start_token_id
                dec.masked_fill_(dec == -100, self.pad_token_id)
                batch["decoder_input_ids"] = dec
        if self.pin_memory and torch.cuda.is_available():
            batch = {k: v.pin_memory() for k, v in batch.items()}
        return batch
