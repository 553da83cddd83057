"""T5 / FLAN-T5 encoder-decoder, written for the fused-op library.

Behaviour follows transformers' T5ForConditionalGeneration (modeling_t5.py:939-1066, the model the
reference fine-tunes through ``AutoModelForSeq2SeqLM``), restructured for MI355X:

* module paths mirror HF (``encoder.block.{i}.layer.{j}.SelfAttention``...) so checkpoints map 1:1,
  but q/k/v (and cross-attention k/v, and gated wi_0/wi_1) are ONE weight each → one GEMM, viewed
  as ``[B, S, 3, H, D]`` by the attention kernel without transposes (models/hf_io.py splits them);
* every residual update ``h + dropout(sublayer)`` is fused with the NEXT sub-layer's RMSNorm
  (ops/norms.py), so the residual stream is read/written once per sub-layer;
* the relative-position bias is a per-head LUT (ops/attention.py) — layer 0 owns the bucket table
  and every layer reuses it (modeling_t5.py:739-740), as in HF; UMT5 (``t5_flavor="umt5"``) gives every
  self-attention layer its own table (modeling_umt5.py UMT5LayerSelfAttention), one LUT per layer;
* LM head + cross-entropy: logits in bf16, CE fused (ops/cross_entropy.py), the
  ``d_model**-0.5`` tied-embedding scale (modeling_t5.py:1044-1045) applied to the decoder output.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import activations, attention as attn_ops, norms
from ..parallel.context import (chunked_attention, chunked_cross_attention, context_parallel_encode,
                                long_sequence_chunk, ring_attention)
from ..ops.ffn import ffn, gated_ffn
from ..ops.cross_entropy import cross_entropy
from ..ops.embedding import embedding
from ..ops.linear import Linear, linear, stacked_linear
from ..ops.lm_head import lm_head_loss, wants_lm_head_loss
from ..ops.rng import default_rng
from .blocks import run_block
from .config import Seq2SeqConfig
from .output import Seq2SeqLMOutput


class T5LayerNorm(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.variance_epsilon = eps


class T5Attention(nn.Module):
    def __init__(self, cfg: Seq2SeqConfig, cross: bool, has_relative_attention_bias: bool, is_decoder: bool):
        super().__init__()
        self.cfg = cfg
        self.cross = cross
        self.is_decoder = is_decoder
        self.n_heads = cfg.num_heads
        self.d_kv = cfg.d_kv
        inner = cfg.inner_dim
        if cross:
            self.q = Linear(cfg.d_model, inner, bias=False)
            self.kv = Linear(cfg.d_model, 2 * inner, bias=False)
        else:
            self.qkv = Linear(cfg.d_model, 3 * inner, bias=False)
        self.o = Linear(inner, cfg.d_model, bias=False)
        self.has_relative_attention_bias = has_relative_attention_bias
        if has_relative_attention_bias:
            self.relative_attention_bias = nn.Embedding(cfg.relative_attention_num_buckets, cfg.num_heads)

    def bias_lut(self, q_len, k_len, q_offset=0):
        return attn_ops.relative_bias_lut(self.relative_attention_bias.weight, q_len, k_len,
                                          bidirectional=not self.is_decoder,
                                          num_buckets=self.cfg.relative_attention_num_buckets,
                                          max_distance=self.cfg.relative_attention_max_distance, q_offset=q_offset)

    def project_kv(self, kv_in):
        B, S, _ = kv_in.shape
        return self.kv(kv_in).view(B, S, 2, self.n_heads, self.d_kv)

    def forward(self, x, kv_in=None, mask=None, lut=None, causal=False, p=0.0, cache=None, kv=None):
        B, S, _ = x.shape
        H, D = self.n_heads, self.d_kv
        seed = default_rng().next_seed() if p > 0 else 0
        kw = dict(scale=1.0, causal=causal, key_padding_mask=mask, bias_lut=lut, dropout_p=p, seed=seed)
        if self.cross:
            q = self.q(x).view(B, S, H, D)
            kv = kv if kv is not None else self.project_kv(kv_in)
            if kv.shape[0] != B:  # beam search: the nb hypotheses of a batch entry share its encoder K/V (read once)
                q = q.reshape(kv.shape[0], (B // kv.shape[0]) * S, H, D)
            chunk = long_sequence_chunk(kv.shape[1], cross=True)
            if chunk is not None:  # long encoder output: key-chunked blocks merged by LSE
                o = chunked_cross_attention(q, kv[:, :, 0], kv[:, :, 1], chunk=chunk, scale=1.0,
                                            key_padding_mask=mask, dropout_p=p, seed=seed)
            else:
                o = attn_ops.attention_q_kv(q, kv, **kw)
        elif isinstance(lut, _CPBias):  # encoder sequence sharded over a CP group: ring attention
            qkv = self.qkv(x).view(B, S, 3, H, D)
            kw2 = dict(scale=1.0, key_padding_mask=mask, bias_table=lut.table, bidirectional=True,
                       num_buckets=self.cfg.relative_attention_num_buckets,
                       max_distance=self.cfg.relative_attention_max_distance, dropout_p=p, seed=seed)
            if lut.chunk is not None:
                o = chunked_attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], chunk=lut.chunk, **kw2)
            else:
                o = ring_attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], group=lut.group, **kw2)
        else:
            qkv = self.qkv(x).view(B, S, 3, H, D)
            if cache is not None:
                k, v = cache.append(qkv[:, :, 1], qkv[:, :, 2])
                o = attn_ops.attention(qkv[:, :, 0], k, v, **kw)
            else:
                o = attn_ops.attention_qkv(qkv, **kw)
        return self.o(o.reshape(B, S, H * D))


class _CPBias:
    """Marker handed to encoder self-attention instead of a bias LUT when the sequence is sharded over a
    context-parallel group (parallel/context.py builds the global-distance LUTs per ring step)."""

    def __init__(self, group, table, chunk=None):
        self.group = group
        self.table = table
        self.chunk = chunk  # set: one device, long sequence in chunk-token blocks (parallel/context.py)


class T5DenseActDense(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.wi = Linear(cfg.d_model, cfg.d_ff * (2 if cfg.is_gated else 1), bias=False)
        self.wo = Linear(cfg.d_ff, cfg.d_model, bias=False)
        self.act = cfg.act
        self.gated = cfg.is_gated

    def forward(self, x, p):
        seed = default_rng().next_seed() if p > 0 else 0
        if not self.gated:  # activation + dropout in the GEMM epilogues where possible (ops/ffn.py)
            return ffn(x, self.wi, self.wo, self.act, p, seed)
        return gated_ffn(x, self.wi, self.wo, self.act, p, seed)


class T5LayerSelfAttention(nn.Module):
    def __init__(self, cfg, has_bias, is_decoder):
        super().__init__()
        self.SelfAttention = T5Attention(cfg, cross=False, has_relative_attention_bias=has_bias, is_decoder=is_decoder)
        self.layer_norm = T5LayerNorm(cfg.d_model, cfg.layer_norm_epsilon)


class T5LayerCrossAttention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.EncDecAttention = T5Attention(cfg, cross=True, has_relative_attention_bias=False, is_decoder=True)
        self.layer_norm = T5LayerNorm(cfg.d_model, cfg.layer_norm_epsilon)


class T5LayerFF(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.DenseReluDense = T5DenseActDense(cfg)
        self.layer_norm = T5LayerNorm(cfg.d_model, cfg.layer_norm_epsilon)


class T5Block(nn.Module):
    def __init__(self, cfg, has_bias, is_decoder):
        super().__init__()
        self.layer = nn.ModuleList([T5LayerSelfAttention(cfg, has_bias, is_decoder)])
        if is_decoder:
            self.layer.append(T5LayerCrossAttention(cfg))
        self.layer.append(T5LayerFF(cfg))

    def norms(self):
        return [lyr.layer_norm for lyr in self.layer]


class T5Stack(nn.Module):
    def __init__(self, cfg: Seq2SeqConfig, is_decoder: bool, embed_tokens: nn.Embedding):
        super().__init__()
        self.cfg = cfg
        self.is_decoder = is_decoder
        self._embed = [embed_tokens]  # shared; not registered twice
        n = cfg.num_decoder_layers if is_decoder else cfg.num_layers
        self.block = nn.ModuleList([T5Block(cfg, has_bias=(i == 0 or cfg.per_layer_position_bias), is_decoder=is_decoder)
                                    for i in range(n)])
        self.final_layer_norm = T5LayerNorm(cfg.d_model, cfg.layer_norm_epsilon)

    def cross_kv_linears(self):
        return [blk.layer[1].EncDecAttention.kv for blk in self.block]

    def project_cross_kv(self, enc_out):
        """All decoder layers' cross-attention K/V in ONE GEMM (ops/linear.py stacked_linear)."""
        B, S, _ = enc_out.shape
        return stacked_linear(enc_out, self.cross_kv_linears(), (B, S, 2, self.cfg.num_heads, self.cfg.d_kv))

    def forward(self, input_ids, attention_mask=None, enc_out=None, enc_mask=None, caches=None, q_offset=0,
                cross_kv=None):
        cfg = self.cfg
        p = cfg.dropout_rate if self.training else 0.0
        pa = cfg.attention_dropout if self.training else 0.0
        eps = cfg.layer_norm_epsilon
        rng = default_rng()
        x = embedding(input_ids, self._embed[0].weight)
        B, S = input_ids.shape
        k_len = S + q_offset
        cp = getattr(self, "_cp_group", False)
        chunk = long_sequence_chunk(S, rows=B * cfg.num_heads) if not self.is_decoder and caches is None else None
        blocks = list(self.block)
        # T5 / mT5: layer 0's table serves every layer; UMT5: each layer's own table
        owners = blocks if cfg.per_layer_position_bias else blocks[:1]
        if (cp is not False or chunk is not None) and not self.is_decoder:
            luts = [_CPBias(cp, b.layer[0].SelfAttention.relative_attention_bias.weight,
                            chunk=chunk if cp is False else None) for b in owners]
        else:
            luts = [b.layer[0].SelfAttention.bias_lut(S, k_len, q_offset=q_offset) for b in owners]
        # h = dropout(embeddings); normed = block0 self-attn norm(h)
        normed, h = norms.dropout_rms_norm(x, blocks[0].layer[0].layer_norm.weight, eps, p,
                                           rng.next_seed() if p > 0 else 0)
        if self.is_decoder and cross_kv is None and enc_out is not None:
            cross_kv = self.project_cross_kv(enc_out)
        for i, blk in enumerate(blocks):
            nxt = blocks[i + 1].layer[0].layer_norm.weight if i + 1 < len(blocks) else self.final_layer_norm.weight
            ckv = cross_kv[i] if cross_kv is not None else None
            cache = caches[i] if caches is not None else None
            lut = luts[i if len(luts) > 1 else 0]

            def run(normed, h, blk=blk, nxt=nxt, ckv=ckv, cache=cache, lut=lut):
                return self._block(blk, nxt, normed, h, attention_mask, lut, enc_out, enc_mask, ckv, cache, p, pa, eps)

            normed, h = run_block(run, normed, h, checkpoint=cfg.gradient_checkpointing and self.training and
                                  caches is None)
        # `normed` is now final_layer_norm(h); HF applies dropout after it (modeling_t5.py:744-745)
        return activations.dropout(normed, p, rng.next_seed() if p > 0 else 0)


    def _block(self, blk, next_norm, normed, h, attention_mask, lut, enc_out, enc_mask, ckv, cache, p, pa, eps):
        """One T5 block on (norm(h), h) -> (next norm(h'), h'): self-attention, [cross-attention], FFN, each
        residual update fused with the following RMSNorm."""
        rng = default_rng()
        subs = list(blk.layer)
        norms_w = [lyr.layer_norm.weight for lyr in subs[1:]] + [next_norm]
        a = subs[0].SelfAttention(normed, mask=attention_mask if not self.is_decoder else None, lut=lut,
                                  causal=self.is_decoder, p=pa, cache=cache)
        normed, h = norms.add_dropout_rms_norm(h, a, norms_w[0], eps, p, rng.next_seed() if p > 0 else 0)
        j = 1
        if self.is_decoder:
            c = subs[1].EncDecAttention(normed, kv_in=enc_out, mask=enc_mask, lut=None, causal=False, p=pa, kv=ckv)
            normed, h = norms.add_dropout_rms_norm(h, c, norms_w[1], eps, p, rng.next_seed() if p > 0 else 0)
            j = 2
        f = subs[j].DenseReluDense(normed, p)
        return norms.add_dropout_rms_norm(h, f, norms_w[j], eps, p, rng.next_seed() if p > 0 else 0)


class T5ForConditionalGeneration(nn.Module):
    model_type = "t5"

    def __init__(self, cfg: Seq2SeqConfig):
        super().__init__()
        self.config = cfg
        self.shared = nn.Embedding(cfg.vocab_size, cfg.d_model)
        self.encoder = T5Stack(cfg, False, self.shared)
        self.decoder = T5Stack(cfg, True, self.shared)
        if not cfg.tie_word_embeddings:
            self.lm_head = Linear(cfg.d_model, cfg.vocab_size, bias=False)
        self.reset_parameters()

    # ---------------------------------------------------------------------------------- init
    @torch.no_grad()
    def reset_parameters(self):
        """HF T5PreTrainedModel._init_weights (modeling_t5.py:563-616)."""
        cfg = self.config
        fac = cfg.initializer_factor
        d, dkv, H, dff = cfg.d_model, cfg.d_kv, cfg.num_heads, cfg.d_ff
        self.shared.weight.normal_(0.0, fac * 1.0)
        if not cfg.tie_word_embeddings:
            self.lm_head.weight.normal_(0.0, fac * 1.0)
        for m in self.modules():
            if isinstance(m, T5LayerNorm):
                m.weight.fill_(fac)
            elif isinstance(m, T5DenseActDense):
                m.wi.weight.normal_(0.0, fac * d ** -0.5)
                m.wo.weight.normal_(0.0, fac * dff ** -0.5)
            elif isinstance(m, T5Attention):
                inner = H * dkv
                if m.cross:
                    m.q.weight.normal_(0.0, fac * (d * dkv) ** -0.5)
                    m.kv.weight.normal_(0.0, fac * d ** -0.5)
                else:
                    m.qkv.weight[:inner].normal_(0.0, fac * (d * dkv) ** -0.5)
                    m.qkv.weight[inner:].normal_(0.0, fac * d ** -0.5)
                m.o.weight.normal_(0.0, fac * (H * dkv) ** -0.5)
                if m.has_relative_attention_bias:
                    m.relative_attention_bias.weight.normal_(0.0, fac * d ** -0.5)

    # ---------------------------------------------------------------------------------- API
    def shift_right(self, labels):
        """modeling_t5.py:618-637"""
        out = labels.new_zeros(labels.shape)
        out[..., 1:] = labels[..., :-1]
        out[..., 0] = self.config.decoder_start_token_id
        out.masked_fill_(out == -100, self.config.pad_token_id)
        return out

    prepare_decoder_input_ids_from_labels = shift_right

    def encode(self, input_ids, attention_mask=None):
        return self.encoder(input_ids, attention_mask=attention_mask)

    def decode(self, decoder_input_ids, enc_out, enc_mask=None, caches=None, q_offset=0, cross_kv=None):
        return self.decoder(decoder_input_ids, enc_out=enc_out, enc_mask=enc_mask, caches=caches, q_offset=q_offset,
                            cross_kv=cross_kv)

    def output_embedding(self):
        return self.shared.weight if self.config.tie_word_embeddings else self.lm_head.weight

    def lm_logits(self, hidden):
        if self.config.scale_decoder_outputs:
            hidden = hidden * (self.config.d_model ** -0.5)
        return linear(hidden, self.output_embedding())

    def logits_bias(self):
        return None

    def cross_attention_modules(self):
        return [blk.layer[1].EncDecAttention for blk in self.decoder.block]

    def project_cross_kv(self, enc_out):
        return self.decoder.project_cross_kv(enc_out)

    def _dllm_param_groups(self):
        return [[m.weight for m in self.decoder.cross_kv_linears()]]

    def generate(self, input_ids, attention_mask=None, **kw):
        from .generation import generate
        return generate(self, input_ids, attention_mask=attention_mask, **kw)

    def gradient_checkpointing_enable(self, enable: bool = True):
        """HF-style switch: recompute every block in backward (activation memory O(1) in depth)."""
        self.config.gradient_checkpointing = bool(enable)
        for st in (self.encoder, self.decoder):
            st.cfg = self.config

    def enable_context_parallel(self, group=None, enable: bool = True):
        """Shard the ENCODER sequence over ``group`` (None = the default group): ``forward`` then takes this
        rank's contiguous slice of ``input_ids`` / ``attention_mask`` (:func:`parallel.context.shard_sequence`)
        and the full decoder batch.  Encoder self-attention becomes ring attention (parallel/context.py); the
        encoder output is all-gathered along the sequence for the decoder, which every CP rank runs on the
        same batch.  The dropout seed stream must be identical on the ranks of one CP group."""
        if enable:
            self.encoder._cp_group = group
        elif hasattr(self.encoder, "_cp_group"):
            del self.encoder._cp_group
        return self

    def forward(self, input_ids=None, attention_mask=None, decoder_input_ids=None, labels=None,
                label_smoothing: float = 0.0, return_logits: bool = False, encoder_outputs=None):
        cp = getattr(self.encoder, "_cp_group", False)
        if cp is not False and encoder_outputs is None:
            enc, attention_mask = context_parallel_encode(self.encode, input_ids, attention_mask, cp)
        else:
            enc = encoder_outputs if encoder_outputs is not None else self.encode(input_ids, attention_mask)
        if decoder_input_ids is None:
            decoder_input_ids = self.shift_right(labels)
        dec = self.decode(decoder_input_ids, enc, attention_mask)
        if labels is not None and not return_logits and wants_lm_head_loss(dec, labels.numel(), self.config.vocab_size):
            # LM head + CE without materialised logits: GEMM-epilogue CE or vocabulary chunks (ops/lm_head.py)
            scale = self.config.d_model ** -0.5 if self.config.scale_decoder_outputs else None
            loss = lm_head_loss(dec, self.output_embedding(), labels, scale=scale, label_smoothing=label_smoothing)
            return Seq2SeqLMOutput(loss=loss, logits=None, encoder_last_hidden_state=enc)
        logits = self.lm_logits(dec)
        loss = None
        if labels is not None:
            V = logits.shape[-1]
            loss = cross_entropy(logits.view(-1, V), labels.reshape(-1), label_smoothing=label_smoothing,
                                 inplace_grad=not return_logits)
        return Seq2SeqLMOutput(loss=loss, logits=logits if (return_logits or labels is None) else None,
                               encoder_last_hidden_state=enc)
