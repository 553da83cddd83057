"""Datasets: SAMSum JSON files, tokenised features, synthetic data.

The reference reads ``train.json`` / ``val.json`` from the Valohai input directory with
``load_dataset('json', ...)`` (ref/train-torchrun.py:150-159) — a JSON array (or JSON lines) of
``{"id", "dialogue", "summary"}`` records — and maps ``convert_examples_to_features`` over it
(ref/train-accelerator.py:114-133): dialogue → ``input_ids``/``attention_mask`` padded to
``max_length`` (1024), summary (``text_target``) → ``labels`` padded to 128 WITH THE PAD ID (so pad
tokens are trained on; SURVEY.md Appendix A Q7 — kept as the default, ``ignore_pad_labels`` opts
out).  Arrow is not needed: features are numpy int32 arrays.
"""
from __future__ import annotations

import json
import os
import random

import numpy as np


def load_json_records(path: str) -> list[dict]:
    with open(path) as f:
        txt = f.read().strip()
    if not txt:
        return []
    if txt[0] == "[":
        return json.loads(txt)
    return [json.loads(line) for line in txt.splitlines() if line.strip()]


def load_samsum(data_dir: str) -> dict[str, list[dict]]:
    return {"train": load_json_records(os.path.join(data_dir, "train.json")),
            "validation": load_json_records(os.path.join(data_dir, "val.json"))}


class Seq2SeqFeatures:
    """Tokenised, fixed-length features (numpy) with the HF ``Dataset`` surface the loops use."""

    def __init__(self, input_ids, attention_mask, labels, records=None):
        self.input_ids = np.asarray(input_ids, dtype=np.int32)
        self.attention_mask = np.asarray(attention_mask, dtype=np.int8)
        self.labels = np.asarray(labels, dtype=np.int32)
        self.records = records

    def __len__(self):
        return len(self.input_ids)

    def __getitem__(self, i):
        return {"input_ids": self.input_ids[i], "attention_mask": self.attention_mask[i], "labels": self.labels[i]}

    @property
    def column_names(self):
        return ["input_ids", "attention_mask", "labels"]


def convert_examples_to_features(records, tokenizer, max_source_length=1024, max_target_length=128,
                                 ignore_pad_labels=False, text_key="dialogue", summary_key="summary"):
    src = tokenizer([r[text_key] for r in records], padding="max_length", truncation=True,
                    max_length=max_source_length)
    tgt = tokenizer(text_target=[r[summary_key] for r in records], padding="max_length", truncation=True,
                    max_length=max_target_length)
    labels = np.asarray(tgt["input_ids"], dtype=np.int32)
    if ignore_pad_labels:
        labels = np.where(np.asarray(tgt["attention_mask"]) == 1, labels, -100)
    return Seq2SeqFeatures(src["input_ids"], src["attention_mask"], labels, records)


class SyntheticSeq2Seq:
    """Random token ids of the SAMSum feature shape (what bench.py and the perf configs train on)."""

    def __init__(self, n: int, src_len: int, tgt_len: int, vocab_size: int, seed: int = 0, pad_frac: float = 0.0,
                 pad_token_id: int = 0):
        rng = np.random.default_rng(seed)
        self.input_ids = rng.integers(3, vocab_size, size=(n, src_len), dtype=np.int32)
        self.attention_mask = np.ones((n, src_len), dtype=np.int8)
        if pad_frac > 0:
            lens = rng.integers(int(src_len * (1 - pad_frac)), src_len + 1, size=n)
            for i, L in enumerate(lens):
                self.attention_mask[i, L:] = 0
                self.input_ids[i, L:] = pad_token_id
        self.labels = rng.integers(3, vocab_size, size=(n, tgt_len), dtype=np.int32)

    def __len__(self):
        return len(self.input_ids)

    def __getitem__(self, i):
        return {"input_ids": self.input_ids[i], "attention_mask": self.attention_mask[i], "labels": self.labels[i]}


_WORDS = ("hey how are you doing today i will be there at five see you soon thanks ok sure what about the meeting "
          "tomorrow can we move it to monday please send me the file love it great idea no problem call me later "
          "dinner movie tonight party weekend train late sorry").split()


def synthetic_samsum_records(n: int, seed: int = 0) -> list[dict]:
    """Text records in the SAMSum schema (CLI smoke tests / offline runs)."""
    r = random.Random(seed)
    names = ["Amanda", "Jerry", "Tom", "Anna", "Kate", "Paul"]
    out = []
    for i in range(n):
        a, b = r.sample(names, 2)
        turns = []
        for t in range(r.randint(2, 8)):
            who = a if t % 2 == 0 else b
            turns.append(f"{who}: " + " ".join(r.choice(_WORDS) for _ in range(r.randint(3, 12))))
        summary = f"{a} and {b} " + " ".join(r.choice(_WORDS) for _ in range(r.randint(4, 12))) + "."
        out.append({"id": f"syn{i:06d}", "dialogue": "\r\n".join(turns), "summary": summary})
    return out


def write_synthetic_samsum(data_dir: str, n_train: int = 64, n_val: int = 16, seed: int = 0):
    os.makedirs(data_dir, exist_ok=True)
    with open(os.path.join(data_dir, "train.json"), "w") as f:
        json.dump(synthetic_samsum_records(n_train, seed), f)
    with open(os.path.join(data_dir, "val.json"), "w") as f:
        json.dump(synthetic_samsum_records(n_val, seed + 1), f)
