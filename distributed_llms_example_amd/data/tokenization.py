"""Tokenizers.

The reference uses ``AutoTokenizer.from_pretrained(model_ckpt)`` (ref/train-torchrun.py:34): BART's
byte-level BPE / T5's SentencePiece, via the Rust ``tokenizers`` library.  That library is installed
and is used whenever the checkpoint directory has tokenizer files.  This box is offline with no cached
vocabularies, so :class:`WordTokenizer` is a self-contained fallback: a word-level vocabulary built
from the training text (most frequent words), with the model's special-token ids, invertible so that
generated ids decode to text for ROUGE.  Both expose the subset of the HF tokenizer API the runtime
uses: ``__call__(texts, max_length, padding, truncation)``, ``text_target=``, ``batch_decode``,
``pad_token_id``, ``save_pretrained``.
"""
from __future__ import annotations

import collections
import json
import os
import re

_WORD = re.compile(r"\w+|[^\w\s]", re.UNICODE)


class WordTokenizer:
    def __init__(self, vocab: list[str], pad_token_id: int = 0, eos_token_id: int = 1, unk_token_id: int = 2,
                 bos_token_id: int | None = None, model_max_length: int = 1024, add_eos: bool = True):
        self.vocab = vocab
        self.index = {w: i for i, w in enumerate(vocab)}
        self.pad_token_id = pad_token_id
        self.eos_token_id = eos_token_id
        self.unk_token_id = unk_token_id
        self.bos_token_id = bos_token_id
        self.model_max_length = model_max_length
        self.add_eos = add_eos
        self.special_ids = {i for i in (pad_token_id, eos_token_id, unk_token_id, bos_token_id) if i is not None}

    @classmethod
    def build(cls, texts, vocab_size: int, pad_token_id=0, eos_token_id=1, unk_token_id=2, bos_token_id=None,
              model_max_length=1024):
        specials = {pad_token_id: "<pad>", eos_token_id: "</s>", unk_token_id: "<unk>"}
        if bos_token_id is not None:
            specials[bos_token_id] = "<s>"
        n_special = max(specials) + 1
        counts = collections.Counter()
        for t in texts:
            counts.update(w.lower() for w in _WORD.findall(t or ""))
        words = [w for w, _ in counts.most_common(max(0, vocab_size - n_special))]
        vocab = [specials.get(i, f"<extra_{i}>") for i in range(n_special)] + words
        return cls(vocab, pad_token_id, eos_token_id, unk_token_id, bos_token_id, model_max_length)

    @property
    def vocab_size(self):
        return len(self.vocab)

    def encode(self, text: str, max_length: int | None = None, truncation: bool = True) -> list[int]:
        ids = [self.index.get(w.lower(), self.unk_token_id) for w in _WORD.findall(text or "")]
        if self.bos_token_id is not None:
            ids = [self.bos_token_id] + ids
        if self.add_eos:
            ids = ids + [self.eos_token_id]
        if truncation and max_length is not None and len(ids) > max_length:
            ids = ids[: max_length - 1] + ([self.eos_token_id] if self.add_eos else [ids[max_length - 1]])
        return ids

    def __call__(self, texts=None, text_target=None, max_length=None, padding=False, truncation=True,
                 return_tensors=None):
        src = texts if texts is not None else text_target
        single = isinstance(src, str)
        src = [src] if single else list(src)
        max_length = max_length or self.model_max_length
        ids = [self.encode(t, max_length, truncation) for t in src]
        if padding == "max_length":
            tgt = max_length
        elif padding in (True, "longest"):
            tgt = max(len(x) for x in ids) if ids else 0
        else:
            tgt = None
        masks = []
        for i, x in enumerate(ids):
            m = [1] * len(x)
            if tgt is not None and len(x) < tgt:
                x = x + [self.pad_token_id] * (tgt - len(x))
                m = m + [0] * (tgt - len(m))
            ids[i] = x
            masks.append(m)
        out = {"input_ids": ids, "attention_mask": masks}
        if return_tensors == "pt":
            import torch
            out = {k: torch.tensor(v) for k, v in out.items()}
        if single:
            out = {k: v[0] for k, v in out.items()}
        return out

    def decode(self, ids, skip_special_tokens: bool = True, **_):
        words = []
        for i in ids:
            i = int(i)
            if i < 0:
                continue
            if skip_special_tokens and i in self.special_ids:
                continue
            words.append(self.vocab[i] if i < len(self.vocab) else "<unk>")
        return " ".join(words)

    def batch_decode(self, batch, skip_special_tokens: bool = True, **kw):
        return [self.decode(x, skip_special_tokens=skip_special_tokens) for x in batch]

    def save_pretrained(self, path: str):
        os.makedirs(path, exist_ok=True)
        with open(os.path.join(path, "word_tokenizer.json"), "w") as f:
            json.dump({"vocab": self.vocab, "pad_token_id": self.pad_token_id, "eos_token_id": self.eos_token_id,
                       "unk_token_id": self.unk_token_id, "bos_token_id": self.bos_token_id,
                       "model_max_length": self.model_max_length}, f)

    @classmethod
    def from_file(cls, path: str):
        with open(path) as f:
            d = json.load(f)
        return cls(d["vocab"], d["pad_token_id"], d["eos_token_id"], d["unk_token_id"], d.get("bos_token_id"),
                   d.get("model_max_length", 1024))


def load_tokenizer(name_or_path: str, cfg, texts=None):
    """HF tokenizer if ``name_or_path`` is a directory with tokenizer files (or the HF cache has it);
    otherwise a :class:`WordTokenizer` fitted on ``texts`` with the model's special-token ids."""
    if name_or_path and os.path.isdir(name_or_path):
        wt = os.path.join(name_or_path, "word_tokenizer.json")
        if os.path.exists(wt):
            return WordTokenizer.from_file(wt)
        if any(os.path.exists(os.path.join(name_or_path, f)) for f in
               ("tokenizer.json", "spiece.model", "vocab.json", "tokenizer_config.json")):
            from transformers import AutoTokenizer
            return AutoTokenizer.from_pretrained(name_or_path)
    unk = 2 if cfg.model_type == "t5" else 3
    return WordTokenizer.build(texts or [], cfg.vocab_size, pad_token_id=cfg.pad_token_id,
                               eos_token_id=cfg.eos_token_id, unk_token_id=unk,
                               bos_token_id=cfg.bos_token_id if cfg.model_type == "bart" else None,
                               model_max_length=1024 if cfg.model_type == "bart" else 512)
