"""Autoregressive generation for the seq2seq models: greedy and beam search with a KV cache.

The reference evaluates with ``unwrap_model(model).generate(input_ids, attention_mask=...,
max_length=128, num_beams=2)`` (ref/train-accelerator.py:239-249, ref/train-task.py:310-313), i.e.
transformers' GenerationMixin beam search (generation/utils.py:3208): encode once, expand to
``batch × num_beams``, per step fp32 ``log_softmax`` + logits processors, top-``2·num_beams``
candidates over ``num_beams × V``, finished hypotheses scored ``sum_logprobs / len**length_penalty``,
``early_stopping`` rules, cache reordering.  Processors implemented: ``min_length``,
``no_repeat_ngram_size``, ``forced_bos_token_id``, ``forced_eos_token_id`` (bart-large-cnn's
generation_config uses all of them).

MI355X specifics: the decoder self-attention cache is preallocated ``[B, max_len, H, D]`` (no
per-step concatenation; the attention kernel reads the strided prefix view), cross-attention K/V are
projected once per generate call, and every decode step runs the same fused kernels as training
(attention with the bias LUT offset by the cache length).
"""
from __future__ import annotations


import torch

from ..ops import routing
from ..ops.attention import relative_bias_lut  # noqa: F401  (documented dependency)


class KVStore:
    """Self-attention K/V of EVERY decoder layer in one preallocated buffer [layers * 2, rows, max_len, H * D].

    A beam reorder is ONE in-place kernel over all layers on the GPU (csrc/beam.hip ``kv_reorder``): a batch entry
    whose hypotheses all kept their own row moves no bytes, and otherwise only the rows that change are written (the
    group's source rows are read first).  That replaces an index_select + copy-back per layer and tensor (48 launches
    and two full passes over the live prefix for a 12-layer decoder)."""

    def __init__(self, layers: int, batch: int, max_len: int, heads: int, dim: int, dtype, device, nb: int = 1):
        self.buf = torch.empty(layers * 2, batch, max_len, heads * dim, dtype=dtype, device=device)
        self.heads, self.dim, self.nb = heads, dim, nb
        self.len = 0
        self.layers = [KVCache(self, i) for i in range(layers)]

    def reorder(self, idx):
        n = self.len
        if not n:
            return
        from .. import _ext
        hd = self.heads * self.dim
        if (self.buf.dtype == torch.bfloat16 and _ext.use_native(self.buf) and self.nb * hd // 8 <= 512
                and hd % 8 == 0):
            _ext.native().kv_reorder(self.buf, idx.contiguous(), self.nb, n)
            return
        live = self.buf[:, :, :n]
        live.copy_(live.index_select(1, idx))


class KVCache:
    """Layer ``i``'s view of a KVStore (the interface the attention modules use: append, then read the prefix)."""

    def __init__(self, store: KVStore, i: int):
        self.store = store
        self.i = i

    @property
    def len(self):
        return self.store.len

    def append(self, k, v):
        st = self.store
        s = k.shape[1]
        last = self.i == len(st.layers) - 1
        kb = st.buf[2 * self.i].view(-1, st.buf.shape[2], st.heads, st.dim)
        vb = st.buf[2 * self.i + 1].view(-1, st.buf.shape[2], st.heads, st.dim)
        kb[:, st.len:st.len + s] = k
        vb[:, st.len:st.len + s] = v
        n = st.len + s
        if last:  # the last layer of the step advances the shared length
            st.len = n
        return kb[:, :n], vb[:, :n]


def _head_geom(model):
    cfg = model.config
    if cfg.model_type == "t5":
        return cfg.num_heads, cfg.d_kv
    return cfg.num_heads, cfg.d_model // cfg.num_heads


def _ban_ngrams(logp, seqs, cur_len: int, n: int):
    """no_repeat_ngram_size on the device: every earlier n-gram whose first n-1 tokens equal the last n-1 generated
    tokens bans its n-th token (transformers NoRepeatNGramLogitsProcessor), without a host round trip."""
    if n <= 0 or cur_len < n:  # no complete earlier n-gram yet
        return logp
    prev = seqs[:, :cur_len]
    if n == 1:
        return logp.scatter_(1, prev, float("-inf"))
    wins = prev.unfold(1, n, 1)  # [N, cur_len - n + 1, n]
    match = (wins[:, :, :n - 1] == prev[:, cur_len - n + 1:cur_len].unsqueeze(1)).all(-1)
    tok = wins[:, :, n - 1]
    vals = torch.where(match, torch.full_like(tok, 0, dtype=logp.dtype) - float("inf"),
                       torch.full_like(tok, 0, dtype=logp.dtype) + float("inf"))
    return logp.scatter_reduce_(1, tok, vals, reduce="amin", include_self=True)


def _apply_processors_device(logp, seqs, cur_len, min_length, no_repeat_ngram_size, forced_bos, forced_eos,
                             max_length, eos):
    """transformers' processor order: NoRepeatNGram and MinLength, then ForcedBOS / ForcedEOS (a forced token wins
    over a ban)."""
    if min_length is not None and cur_len < min_length and eos is not None:
        logp[:, eos] = -float("inf")
    logp = _ban_ngrams(logp, seqs, cur_len, no_repeat_ngram_size or 0)
    if forced_bos is not None and cur_len == 1:
        logp.fill_(-float("inf"))
        logp[:, forced_bos] = 0.0
    if forced_eos is not None and cur_len == max_length - 1:
        logp.fill_(-float("inf"))
        logp[:, forced_eos] = 0.0
    return logp


def _fused_beam_ok(logits, nb: int) -> bool:
    from .. import _ext
    return (bool(routing.get("gen_fused_beam")) and nb <= 8 and 2 * nb <= 16 and logits.dim() == 2
            and logits.dtype in (torch.bfloat16, torch.float32) and _ext.use_native(logits))


def _beam_candidates(logits, beam_scores, seqs, cur, B, nb, proc):
    """Top-2·nb candidates over nb·V per batch entry: (scores [B, 2nb], flat indices beam·V + token).  On the GPU one
    csrc/beam.hip launch (log_softmax normaliser + processors + beam score + top-k in one pass over the logits);
    otherwise the torch composite of the same ops."""
    min_length, ngram, forced_bos, forced_eos, max_length, eos = proc
    if _fused_beam_ok(logits, nb):
        from .. import _ext
        ban = eos if (min_length is not None and cur < min_length and eos is not None) else -1
        force = -1
        if forced_bos is not None and cur == 1:
            force = forced_bos
        if forced_eos is not None and cur == max_length - 1:
            force = forced_eos
        top_s, top_i = _ext.native().beam_topk(logits.contiguous(), beam_scores.reshape(-1).float().contiguous(), seqs,
                                               cur, ngram or 0, ban, force, nb, 2 * nb)
        return top_s, top_i
    logp = _apply_processors_device(torch.log_softmax(logits.float(), dim=-1), seqs, cur, min_length, ngram,
                                    forced_bos, forced_eos, max_length, eos)
    V = logp.shape[-1]
    return (beam_scores.view(-1, 1) + logp).view(B, nb * V).topk(2 * nb, dim=1)


def _apply_processors(logp, seqs, cur_len, cfg, min_length, no_repeat_ngram_size, forced_bos, forced_eos,
                      max_length, eos):
    V = logp.shape[-1]
    if min_length is not None and cur_len < min_length and eos is not None:
        logp[:, eos] = -float("inf")
    n = no_repeat_ngram_size or 0
    if n > 0 and cur_len + 1 >= n:  # bans before the forced tokens (transformers' order: a forced token wins)
        rows = seqs.tolist()
        for b, row in enumerate(rows):
            prefix = tuple(row[cur_len - n + 1:cur_len]) if n > 1 else ()
            banned = set()
            for i in range(cur_len - n + 1):
                if tuple(row[i:i + n - 1]) == prefix:
                    banned.add(row[i + n - 1])
            if banned:
                logp[b, [t for t in banned if t < V]] = -float("inf")
    if forced_bos is not None and cur_len == 1:
        logp[:] = -float("inf")
        logp[:, forced_bos] = 0.0
    if forced_eos is not None and cur_len == max_length - 1:
        logp[:] = -float("inf")
        logp[:, forced_eos] = 0.0
    return logp


def _beam_search_device(model, seqs, enc, attention_mask, caches, cross, B, nb, max_length, proc, eos, pad,
                        length_penalty, early_stopping, check_every):
    """Beam search with all bookkeeping on the device (transformers BeamSearchScorer semantics): top-2·nb candidates
    over nb·V, eos candidates ranked < nb scored ``sum_logprobs / len**length_penalty`` into a per-batch top-nb of
    finished hypotheses, the first nb non-eos candidates become the next beams, ``is_done`` per batch; the host only
    looks at ``done.all()`` every ``check_every`` steps and at the final length."""
    dev = seqs.device
    L = max_length
    inf = float("inf")
    beam_scores = torch.zeros(B, nb, device=dev)
    beam_scores[:, 1:] = -1e9
    fin_scores = torch.full((B, nb), -inf, device=dev)
    fin_seqs = torch.full((B, nb, L), pad, dtype=torch.long, device=dev)
    fin_len = torch.zeros(B, nb, dtype=torch.long, device=dev)
    fin_cnt = torch.zeros(B, dtype=torch.long, device=dev)
    done = torch.zeros(B, dtype=torch.bool, device=dev)
    base = torch.arange(B, device=dev).unsqueeze(1) * nb
    rank = torch.arange(2 * nb, device=dev).unsqueeze(0)

    def add_finished(scores, cand_seqs, cand_len):
        nonlocal fin_scores, fin_seqs, fin_len
        all_s = torch.cat([fin_scores, scores], 1)
        keep_s, keep_i = all_s.topk(nb, dim=1)
        all_seq = torch.cat([fin_seqs, cand_seqs], 1)
        fin_seqs = all_seq.gather(1, keep_i.unsqueeze(-1).expand(-1, -1, L))
        fin_len = torch.cat([fin_len, cand_len], 1).gather(1, keep_i)
        fin_scores = keep_s

    cur = 1
    while cur < max_length:
        h = model.decode(seqs[:, cur - 1:cur], enc, attention_mask, caches=caches, q_offset=cur - 1, cross_kv=cross)
        logits = model.lm_logits(h[:, -1])
        V = logits.shape[-1]
        top_s, top_i = _beam_candidates(logits, beam_scores, seqs, cur, B, nb, proc)
        src = base + top_i // V
        tok = top_i % V
        is_eos = tok == eos if eos is not None else torch.zeros_like(tok, dtype=torch.bool)
        # finished hypotheses: eos candidates among the top nb of a live batch
        add = is_eos & (rank < nb) & ~done.unsqueeze(1)
        if eos is not None:
            sc = torch.where(add, top_s / (max(cur, 1) ** length_penalty), torch.full_like(top_s, -inf))
            cand = seqs.index_select(0, src.reshape(-1)).view(B, 2 * nb, L)
            cand[:, :, cur] = tok
            add_finished(sc, cand, torch.full_like(tok, cur + 1))
            fin_cnt = torch.clamp(fin_cnt + add.sum(1), max=nb)
        # next beams: the first nb non-eos candidates in rank order; finished batches stay frozen on pad
        order = (is_eos.long() * (2 * nb) + rank).argsort(dim=1)[:, :nb]
        new_scores = top_s.gather(1, order)
        new_src = src.gather(1, order)
        new_tok = tok.gather(1, order)
        dn = done.unsqueeze(1)
        new_scores = torch.where(dn, torch.full_like(new_scores, -1e9), new_scores)
        new_src = torch.where(dn, base.expand(-1, nb), new_src)
        new_tok = torch.where(dn, torch.full_like(new_tok, pad), new_tok)
        # BeamHypotheses.is_done
        full = fin_cnt >= nb
        if early_stopping is True:
            now = full
        else:
            gl = cur if early_stopping is False else max_length - 1
            now = full & (fin_scores.min(1).values >= new_scores.max(1).values / (max(gl, 1) ** length_penalty))
        done = done | now
        idx = new_src.reshape(-1)
        seqs = seqs.index_select(0, idx)
        seqs[:, cur] = new_tok.reshape(-1)
        caches[0].store.reorder(idx)
        beam_scores = new_scores
        cur += 1
        if cur % check_every == 0 and bool(done.all()):
            break
    # finalize: the running beams of unfinished batches join the finished hypotheses, best one per batch
    live = ~done.unsqueeze(1)
    sc = torch.where(live, beam_scores / (max(cur - 1, 1) ** length_penalty), torch.full_like(beam_scores, -inf))
    add_finished(sc, seqs.view(B, nb, L), torch.full((B, nb), cur, dtype=torch.long, device=dev))
    best, best_len = fin_seqs[:, 0], fin_len[:, 0]
    return best[:, :int(best_len.max())]


@torch.no_grad()
def generate(model, input_ids, attention_mask=None, max_length: int | None = None, num_beams: int | None = None,
             min_length: int | None = None, length_penalty: float | None = None, no_repeat_ngram_size=None,
             early_stopping=None, forced_bos_token_id=None, forced_eos_token_id=None, max_new_tokens=None,
             **_unused):
    cfg = model.config
    gen = dict(cfg.generation)
    max_length = max_length if max_length is not None else gen.get("max_length", 20)
    if max_new_tokens is not None:
        max_length = max_new_tokens + 1
    num_beams = num_beams if num_beams is not None else gen.get("num_beams", 1)
    min_length = min_length if min_length is not None else gen.get("min_length", 0)
    length_penalty = length_penalty if length_penalty is not None else gen.get("length_penalty", 1.0)
    no_repeat_ngram_size = no_repeat_ngram_size if no_repeat_ngram_size is not None else \
        gen.get("no_repeat_ngram_size", 0)
    early_stopping = early_stopping if early_stopping is not None else gen.get("early_stopping", False)
    forced_bos = forced_bos_token_id if forced_bos_token_id is not None else cfg.forced_bos_token_id
    forced_eos = forced_eos_token_id if forced_eos_token_id is not None else cfg.forced_eos_token_id
    eos, pad, start = cfg.eos_token_id, cfg.pad_token_id, cfg.decoder_start_token_id
    was_training = model.training
    model.eval()
    try:
        B = input_ids.shape[0]
        dev = input_ids.device
        enc = model.encode(input_ids, attention_mask)
        nb = max(1, num_beams)
        # cross-attention K/V projected once per batch entry and shared by its nb hypotheses: the decoder's
        # cross-attention runs the beams as nb query rows of one (entry, head) — K/V read once per step, not nb times
        cross = model.project_cross_kv(enc)
        if nb > 1 and not routing.get("gen_shared_cross"):  # A/B: per-hypothesis copies
            enc = enc.repeat_interleave(nb, 0)
            attention_mask = attention_mask.repeat_interleave(nb, 0) if attention_mask is not None else None
            cross = model.project_cross_kv(enc)
        N = B * nb
        H, D = _head_geom(model)
        dtype = next(model.parameters()).dtype
        store = KVStore(cfg.num_decoder_layers, N, max_length, H, D, dtype, dev, nb)
        caches = store.layers
        seqs = torch.full((N, max_length), pad, dtype=torch.long, device=dev)
        seqs[:, 0] = start
        cur = 1
        check_every = max(1, int(routing.get("gen_check_every")))

        def process(logp, sq, c):
            return _apply_processors_device(logp, sq, c, min_length, no_repeat_ngram_size, forced_bos, forced_eos,
                                            max_length, eos)

        if nb == 1:  # greedy: device-side done flags, one host check every check_every steps
            done = torch.zeros(B, dtype=torch.bool, device=dev)
            all_done_at = []
            while cur < max_length:
                h = model.decode(seqs[:, cur - 1:cur], enc, attention_mask, caches=caches, q_offset=cur - 1,
                                 cross_kv=cross)
                logp = process(torch.log_softmax(model.lm_logits(h[:, -1]).float(), dim=-1), seqs, cur)
                nxt = logp.argmax(-1)
                nxt = torch.where(done, torch.full_like(nxt, pad), nxt)
                seqs[:, cur] = nxt
                if eos is not None:
                    done |= nxt == eos
                all_done_at.append(done.all())
                cur += 1
                if cur % check_every == 0 and bool(all_done_at[-1]):
                    break
            # trim the steps run after every sequence had finished (at most check_every - 1)
            flags = torch.stack(all_done_at).tolist() if all_done_at else []
            end = next((i + 2 for i, f in enumerate(flags) if f), cur)
            return seqs[:, :end]
        if not routing.get("gen_host"):
            proc = (min_length, no_repeat_ngram_size, forced_bos, forced_eos, max_length, eos)
            return _beam_search_device(model, seqs, enc, attention_mask, caches, cross, B, nb, max_length, proc,
                                       eos, pad, length_penalty, early_stopping, check_every)
        # ---------------------------------------------------------------- beam search, host bookkeeping
        # (routing gen_host=1: the original per-step host loop, kept as the A/B oracle of the device version)
        beam_scores = torch.zeros(B, nb, device=dev)
        beam_scores[:, 1:] = -1e9
        beam_scores = beam_scores.view(-1)
        finished = [[] for _ in range(B)]  # (score, tokens)
        batch_done = [False] * B
        V = cfg.vocab_size
        while cur < max_length:
            h = model.decode(seqs[:, cur - 1:cur], enc, attention_mask, caches=caches, q_offset=cur - 1,
                             cross_kv=cross)
            logp = torch.log_softmax(model.lm_logits(h[:, -1]).float(), dim=-1)
            logp = _apply_processors(logp, seqs[:, :cur], cur, cfg, min_length, no_repeat_ngram_size, forced_bos,
                                     forced_eos, max_length, eos)
            V = logp.shape[-1]
            cand = (beam_scores[:, None] + logp).view(B, nb * V)
            top_s, top_i = cand.topk(2 * nb, dim=1)
            top_s, top_i = top_s.tolist(), top_i.tolist()
            new_scores = torch.empty(B, nb, device=dev)
            new_beam = torch.empty(B, nb, dtype=torch.long)
            new_tok = torch.empty(B, nb, dtype=torch.long)
            for b in range(B):
                if batch_done[b]:
                    new_scores[b] = -1e9
                    new_beam[b] = b * nb
                    new_tok[b] = pad
                    continue
                k = 0
                for rank, (s, idx) in enumerate(zip(top_s[b], top_i[b])):
                    beam, tok = divmod(idx, V)
                    src = b * nb + beam
                    if eos is not None and tok == eos:
                        if rank >= nb:
                            continue
                        hyp = seqs[src, :cur].tolist() + [tok]
                        gen_len = len(hyp) - 1
                        finished[b].append((s / (max(gen_len, 1) ** length_penalty), hyp))
                        finished[b].sort(key=lambda x: -x[0])
                        del finished[b][nb:]
                    else:
                        new_scores[b, k] = s
                        new_beam[b, k] = src
                        new_tok[b, k] = tok
                        k += 1
                    if k == nb:
                        break
                # stopping rule (BeamHypotheses.is_done)
                if len(finished[b]) == nb:
                    if early_stopping is True:
                        batch_done[b] = True
                    else:
                        best_running = float(new_scores[b].max())
                        gl = cur if early_stopping is False else max_length - 1
                        if finished[b][-1][0] >= best_running / (max(gl, 1) ** length_penalty):
                            batch_done[b] = True
            beam_idx = new_beam.view(-1).to(dev)
            seqs = seqs.index_select(0, beam_idx)
            seqs[:, cur] = new_tok.view(-1).to(dev)
            caches[0].store.reorder(beam_idx)
            beam_scores = new_scores.view(-1)
            cur += 1
            if all(batch_done):
                break
        # finalize: add running beams
        scores = beam_scores.view(B, nb).tolist()
        for b in range(B):
            if batch_done[b]:
                continue
            for j in range(nb):
                hyp = seqs[b * nb + j, :cur].tolist()
                gen_len = len(hyp) - 1
                finished[b].append((scores[b][j] / (max(gen_len, 1) ** length_penalty), hyp))
            finished[b].sort(key=lambda x: -x[0])
        best = [finished[b][0][1] for b in range(B)]
        L = max(len(x) for x in best)
        out = torch.full((B, L), pad, dtype=torch.long, device=dev)
        for b, x in enumerate(best):
            out[b, : len(x)] = torch.tensor(x, device=dev)
        return out
    finally:
        model.train(was_training)
