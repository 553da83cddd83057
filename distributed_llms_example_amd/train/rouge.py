"""ROUGE-1/2/L/Lsum (F-measure), replacing ``evaluate.load("rouge")`` → ``rouge_score`` (not installed).

Used like the reference (ref/train-accelerator.py:207,266-268): ``metric.add_batch(predictions,
references)`` then ``metric.compute(use_stemmer=True)``.  Tokenisation follows rouge_score: lowercase,
non ``[a-z0-9]`` → space, split, Porter-stem tokens longer than 3 characters.  rougeLsum splits on
newlines and uses the union-LCS summary-level score.  Aggregation is the mean F-measure over samples
(rouge_score's BootstrapAggregator reports a bootstrap "mid" estimate of that same mean).  The
stemmer is the original Porter (1980) algorithm; NLTK's extensions differ on a few irregular words
(parity with rouge_score's nltk stemmer is "unpinned" for those: no reference outputs exist here).
"""
from __future__ import annotations

import collections
import re

_NON_ALNUM = re.compile(r"[^a-z0-9]+")
_VALID = re.compile(r"^[a-z0-9]+$")


# ------------------------------------------------------------------------------------ Porter stemmer
class PorterStemmer:
    vowels = set("aeiou")

    def _cons(self, w, i):
        c = w[i]
        if c in self.vowels:
            return False
        if c == "y":
            return i == 0 or not self._cons(w, i - 1)
        return True

    def _m(self, w):
        n, i, L = 0, 0, len(w)
        while i < L and self._cons(w, i):
            i += 1
        while i < L:
            while i < L and not self._cons(w, i):
                i += 1
            if i >= L:
                break
            n += 1
            while i < L and self._cons(w, i):
                i += 1
        return n

    def _has_vowel(self, w):
        return any(not self._cons(w, i) for i in range(len(w)))

    def _dbl(self, w):
        return len(w) >= 2 and w[-1] == w[-2] and self._cons(w, len(w) - 1)

    def _cvc(self, w):
        if len(w) < 3:
            return False
        return (self._cons(w, len(w) - 3) and not self._cons(w, len(w) - 2) and self._cons(w, len(w) - 1)
                and w[-1] not in "wxy")

    def _rep(self, w, suf, rep, cond=None):
        if w.endswith(suf):
            stem = w[: len(w) - len(suf)]
            if cond is None or cond(stem):
                return stem + rep, True
            return w, True
        return w, False

    def stem(self, w):
        if len(w) <= 2:
            return w
        # step 1a
        if w.endswith("sses"):
            w = w[:-2]
        elif w.endswith("ies"):
            w = w[:-2]
        elif w.endswith("ss"):
            pass
        elif w.endswith("s"):
            w = w[:-1]
        # step 1b
        flag = False
        if w.endswith("eed"):
            if self._m(w[:-3]) > 0:
                w = w[:-1]
        elif w.endswith("ed") and self._has_vowel(w[:-2]):
            w, flag = w[:-2], True
        elif w.endswith("ing") and self._has_vowel(w[:-3]):
            w, flag = w[:-3], True
        if flag:
            if w.endswith(("at", "bl", "iz")):
                w += "e"
            elif self._dbl(w) and w[-1] not in "lsz":
                w = w[:-1]
            elif self._m(w) == 1 and self._cvc(w):
                w += "e"
        # step 1c
        if w.endswith("y") and self._has_vowel(w[:-1]):
            w = w[:-1] + "i"
        m0 = lambda s: self._m(s) > 0  # noqa: E731
        for suf, rep in (("ational", "ate"), ("tional", "tion"), ("enci", "ence"), ("anci", "ance"),
                         ("izer", "ize"), ("abli", "able"), ("alli", "al"), ("entli", "ent"), ("eli", "e"),
                         ("ousli", "ous"), ("ization", "ize"), ("ation", "ate"), ("ator", "ate"), ("alism", "al"),
                         ("iveness", "ive"), ("fulness", "ful"), ("ousness", "ous"), ("aliti", "al"),
                         ("iviti", "ive"), ("biliti", "ble")):
            w, hit = self._rep(w, suf, rep, m0)
            if hit:
                break
        for suf, rep in (("icate", "ic"), ("ative", ""), ("alize", "al"), ("iciti", "ic"), ("ical", "ic"),
                         ("ful", ""), ("ness", "")):
            w, hit = self._rep(w, suf, rep, m0)
            if hit:
                break
        m1 = lambda s: self._m(s) > 1  # noqa: E731
        for suf in ("al", "ance", "ence", "er", "ic", "able", "ible", "ant", "ement", "ment", "ent", "ion", "ou",
                    "ism", "ate", "iti", "ous", "ive", "ize"):
            if w.endswith(suf):
                stem = w[: len(w) - len(suf)]
                if suf == "ion":
                    if m1(stem) and stem and stem[-1] in "st":
                        w = stem
                elif m1(stem):
                    w = stem
                break
        if w.endswith("e"):
            stem = w[:-1]
            m = self._m(stem)
            if m > 1 or (m == 1 and not self._cvc(stem)):
                w = stem
        if self._m(w) > 1 and self._dbl(w) and w.endswith("l"):
            w = w[:-1]
        return w


_stemmer = PorterStemmer()


def tokenize(text: str, use_stemmer: bool) -> list[str]:
    toks = _NON_ALNUM.sub(" ", text.lower()).split()
    if use_stemmer:
        toks = [_stemmer.stem(t) if len(t) > 3 else t for t in toks]
    return [t for t in toks if _VALID.match(t)]


# ------------------------------------------------------------------------------------ scores
def _f(p, r):
    return 0.0 if p + r == 0 else 2 * p * r / (p + r)


def _ngrams(toks, n):
    return collections.Counter(tuple(toks[i:i + n]) for i in range(len(toks) - n + 1))


def rouge_n(pred, ref, n):
    pc, rc = _ngrams(pred, n), _ngrams(ref, n)
    overlap = sum((pc & rc).values())
    p = overlap / max(sum(pc.values()), 1)
    r = overlap / max(sum(rc.values()), 1)
    return _f(p, r)


def _lcs_table(a, b):
    t = [[0] * (len(b) + 1) for _ in range(len(a) + 1)]
    for i in range(1, len(a) + 1):
        ai = a[i - 1]
        row, prev = t[i], t[i - 1]
        for j in range(1, len(b) + 1):
            row[j] = prev[j - 1] + 1 if ai == b[j - 1] else max(prev[j], row[j - 1])
    return t


def rouge_l(pred, ref):
    if not pred or not ref:
        return 0.0
    lcs = _lcs_table(ref, pred)[-1][-1]
    return _f(lcs / len(pred), lcs / len(ref))


def _lcs_indices(ref, cand):
    t = _lcs_table(ref, cand)
    i, j, out = len(ref), len(cand), []
    while i > 0 and j > 0:
        if ref[i - 1] == cand[j - 1]:
            out.append(i - 1)
            i -= 1
            j -= 1
        elif t[i - 1][j] >= t[i][j - 1]:
            i -= 1
        else:
            j -= 1
    return out


def rouge_lsum(pred_sents, ref_sents):
    ref_tokens = sum(len(s) for s in ref_sents)
    cand_tokens = sum(len(s) for s in pred_sents)
    if ref_tokens == 0 or cand_tokens == 0:
        return 0.0
    cr = collections.Counter(t for s in ref_sents for t in s)
    cc = collections.Counter(t for s in pred_sents for t in s)
    hits = 0
    for r in ref_sents:
        union = set()
        for c in pred_sents:
            union.update(_lcs_indices(r, c))
        for i in sorted(union):
            t = r[i]
            if cc[t] > 0 and cr[t] > 0:
                hits += 1
                cc[t] -= 1
                cr[t] -= 1
    return _f(hits / cand_tokens, hits / ref_tokens)


def score(prediction: str, reference: str, use_stemmer: bool = True) -> dict:
    p, r = tokenize(prediction, use_stemmer), tokenize(reference, use_stemmer)
    ps = [tokenize(s, use_stemmer) for s in prediction.split("\n")]
    rs = [tokenize(s, use_stemmer) for s in reference.split("\n")]
    return {"rouge1": rouge_n(p, r, 1), "rouge2": rouge_n(p, r, 2), "rougeL": rouge_l(p, r),
            "rougeLsum": rouge_lsum([s for s in ps if s], [s for s in rs if s])}


class Rouge:
    """``evaluate``-style accumulator."""

    def __init__(self):
        self.preds, self.refs = [], []

    def add_batch(self, predictions, references):
        self.preds.extend(predictions)
        self.refs.extend(references)

    def compute(self, use_stemmer: bool = True) -> dict:
        keys = ("rouge1", "rouge2", "rougeL", "rougeLsum")
        if not self.preds:
            return {k: 0.0 for k in keys}
        tot = dict.fromkeys(keys, 0.0)
        for p, r in zip(self.preds, self.refs):
            s = score(p, r, use_stemmer)
            for k in keys:
                tot[k] += s[k]
        n = len(self.preds)
        self.preds, self.refs = [], []
        return {k: v / n for k, v in tot.items()}


def load(name: str = "rouge") -> Rouge:
    if name != "rouge":
        raise ValueError(name)
    return Rouge()
