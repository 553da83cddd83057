"""Test-set summarisation scoring (the reference's unused ``generate_batch_sized_chunks`` /
``calculate_metric_on_test_ds`` helpers, ref/train-torchrun.py:60-96), made usable.

Same defaults as the reference — CNN/DailyMail-style ``article`` / ``highlights`` columns, inputs truncated and
padded to 1024 tokens, beam search with 8 beams, ``length_penalty`` 0.8, ``max_length`` 128 — with its
no-op ``d.replace("", " ")`` dropped (it inserts a space between every character).  Generation runs on the
framework's own KV-cached beam search (models/generation.py); ROUGE is train/rouge.py.
"""
from __future__ import annotations

from typing import Iterable, Iterator, Sequence

import torch

from . import rouge as rouge_mod


def generate_batch_sized_chunks(items: Sequence, batch_size: int) -> Iterator[Sequence]:
    """Yield successive ``batch_size`` slices of ``items``."""
    for i in range(0, len(items), batch_size):
        yield items[i:i + batch_size]


@torch.no_grad()
def calculate_metric_on_test_ds(model, tokenizer, dataset, metric=None, *, batch_size: int = 8,
                                column_text: str = "article", column_summary: str = "highlights",
                                max_source_length: int = 1024, num_beams: int = 8, length_penalty: float = 0.8,
                                max_length: int = 128, device=None):
    """Generate a summary for every row of ``dataset`` (dict of columns or list of dicts) and score it."""
    if isinstance(dataset, dict):
        texts, refs = list(dataset[column_text]), list(dataset[column_summary])
    else:
        texts = [r[column_text] for r in dataset]
        refs = [r[column_summary] for r in dataset]
    metric = metric if metric is not None else rouge_mod.load("rouge")
    device = device or next(model.parameters()).device
    was_training = model.training
    model.eval()
    for art, ref in zip(generate_batch_sized_chunks(texts, batch_size), generate_batch_sized_chunks(refs, batch_size)):
        enc = tokenizer(list(art), max_length=max_source_length, truncation=True, padding="max_length",
                        return_tensors="pt")
        out = model.generate(enc["input_ids"].to(device), attention_mask=enc["attention_mask"].to(device),
                             num_beams=num_beams, length_penalty=length_penalty, max_length=max_length)
        preds = [tokenizer.decode(s, skip_special_tokens=True, clean_up_tokenization_spaces=True) for s in out]
        metric.add_batch(predictions=preds, references=list(ref))
    model.train(was_training)
    return metric.compute()


def iter_chunks(items: Iterable, batch_size: int) -> Iterator[list]:
    """Chunk an arbitrary iterable (not only sequences)."""
    buf = []
    for x in items:
        buf.append(x)
        if len(buf) == batch_size:
            yield buf
            buf = []
    if buf:
        yield buf
