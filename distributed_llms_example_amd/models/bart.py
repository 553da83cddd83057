"""BART (bart-large-cnn, the reference's default checkpoint: ref/valohai.yaml:10,36,65) and the other
BART-family models ``AutoModelForSeq2SeqLM`` resolves to: mBART, Pegasus, Marian, M2M100 / NLLB, PLBart, Blenderbot.

Follows transformers' BartForConditionalGeneration (modeling_bart.py:835-958): learned positions
with offset 2 (:74-98), ``layernorm_embedding`` + dropout after the embeddings (:507-549),
post-LN encoder/decoder layers (:280-308, :343-390), exact-erf GELU, attention scale d**-0.5
(:169), tied LM head + ``final_logits_bias`` (:939-940).  MI355X restructuring as in models/t5.py:
fused QKV / cross-KV projections (one GEMM each), ``LN(residual + dropout(x))`` as one kernel,
flash attention with key-padding / causal masks, fused CE with the logits bias inside the kernel.
LayerDrop (encoder/decoder_layerdrop, 0.0 in every public BART config) is not implemented.

Family switches (models/config.py ``_FAMILY``; transformers modeling_mbart.py, modeling_pegasus.py,
modeling_marian.py): pre-LN layers plus a final LayerNorm per stack (mBART, Pegasus) — there the residual update
and the NEXT sub-layer's LayerNorm are one kernel returning both (as T5's RMSNorm blocks); no embedding LayerNorm
(Pegasus, Marian, M2M100); fixed sinusoidal positions without offset (Pegasus, Marian; sin in the first half of the
features, cos in the second) or padding-aware with offset 2 (M2M100 / NLLB); SiLU FFN (Marian's ``swish``); no
``final_logits_bias`` (M2M100); learned positions without the offset 2 (Blenderbot); mBART's and PLBart's decoder
input starts from the label's last non-pad token (the language id).
"""
from __future__ import annotations


import math

import torch
import torch.nn as nn

from ..ops import activations, attention as attn_ops, norms
from ..ops.ffn import ffn, ffn_res
from ..ops.cross_entropy import cross_entropy
from ..ops.embedding import embedding
from ..ops.linear import Linear, linear, linear_res, stacked_linear
from ..ops.lm_head import lm_head_loss, wants_lm_head_loss
from ..ops.rng import default_rng
from .blocks import run_block
from .config import Seq2SeqConfig
from .output import Seq2SeqLMOutput


_NORM_BIAS_COLSUM = True  # False: a separate column-sum pass for the out_proj / fc2 bias gradients (tests flip it)

class BartAttention(nn.Module):
    def __init__(self, cfg: Seq2SeqConfig, cross: bool):
        super().__init__()
        d = cfg.d_model
        self.cross = cross
        self.n_heads = cfg.num_heads
        self.head_dim = d // cfg.num_heads
        self.scaling = self.head_dim ** -0.5
        if cross:
            self.q_proj = Linear(d, d)
            self.kv_proj = Linear(d, 2 * d)
        else:
            self.qkv_proj = Linear(d, 3 * d)
        self.out_proj = Linear(d, d)

    def project_kv(self, kv_in):
        B, S, _ = kv_in.shape
        return self.kv_proj(kv_in).view(B, S, 2, self.n_heads, self.head_dim)

    def forward(self, x, kv_in=None, mask=None, causal=False, p=0.0, cache=None, kv=None, residual=False):
        """Attention block output; with ``residual`` also ``x`` for the post-LN residual, its gradient accumulated by
        the input projection's dgrad GEMM (ops/linear.py linear_res)."""
        B, S, _ = x.shape
        res = x
        H, D = self.n_heads, self.head_dim
        seed = default_rng().next_seed() if p > 0 else 0
        kw = dict(scale=self.scaling, causal=causal, key_padding_mask=mask, dropout_p=p, seed=seed)
        if self.cross:
            if residual:
                q, res = linear_res(x, self.q_proj)
                q = q.view(B, S, H, D)
            else:
                q = self.q_proj(x).view(B, S, H, D)
            kv = kv if kv is not None else self.project_kv(kv_in)
            if kv.shape[0] != B:  # beam search: the nb hypotheses of a batch entry share its encoder K/V (read once)
                q = q.reshape(kv.shape[0], (B // kv.shape[0]) * S, H, D)
            o = attn_ops.attention_q_kv(q, kv, **kw)
        else:
            if residual:
                qkv, res = linear_res(x, self.qkv_proj)
                qkv = qkv.view(B, S, 3, H, D)
            else:
                qkv = self.qkv_proj(x).view(B, S, 3, H, D)
            if cache is not None:
                k, v = cache.append(qkv[:, :, 1], qkv[:, :, 2])
                o = attn_ops.attention(qkv[:, :, 0], k, v, **kw)
            else:
                o = attn_ops.attention_qkv(qkv, **kw)
        out = self.out_proj(o.reshape(B, S, H * D))
        return (out, res) if residual else out


class BartLayer(nn.Module):
    def __init__(self, cfg, is_decoder):
        super().__init__()
        d = cfg.d_model
        self.is_decoder = is_decoder
        self.self_attn = BartAttention(cfg, cross=False)
        self.self_attn_layer_norm = nn.LayerNorm(d)
        if is_decoder:
            self.encoder_attn = BartAttention(cfg, cross=True)
            self.encoder_attn_layer_norm = nn.LayerNorm(d)
        self.fc1 = Linear(d, cfg.d_ff)
        self.fc2 = Linear(cfg.d_ff, d)
        self.final_layer_norm = nn.LayerNorm(d)
        self.cfg = cfg

    def forward(self, h, mask=None, enc_out=None, enc_mask=None, cache=None, cross_kv=None):
        cfg = self.cfg
        tr = self.training
        p = cfg.dropout_rate if tr else 0.0
        pa = cfg.attention_dropout if tr else 0.0
        pact = cfg.activation_dropout if tr else 0.0
        eps = cfg.layer_norm_epsilon
        rng = default_rng()
        # post-LN blocks: each block's input is both the sublayer input and the residual; the sublayers hand the
        # residual back from their input projection so its gradient is summed inside that projection's dgrad GEMM
        a, h = self.self_attn(h, mask=None if self.is_decoder else mask, causal=self.is_decoder, p=pa, cache=cache,
                              residual=True)
        xb = _NORM_BIAS_COLSUM  # out_proj / fc2 bias gradients summed by the norm backward kernel (ops/norms.py)
        h = norms.add_dropout_layer_norm(h, a, self.self_attn_layer_norm.weight, self.self_attn_layer_norm.bias, eps,
                                         p, rng.next_seed() if p > 0 else 0, xb)
        if self.is_decoder:
            c, h = self.encoder_attn(h, kv_in=enc_out, mask=enc_mask, p=pa, kv=cross_kv, residual=True)
            h = norms.add_dropout_layer_norm(h, c, self.encoder_attn_layer_norm.weight,
                                             self.encoder_attn_layer_norm.bias, eps, p,
                                             rng.next_seed() if p > 0 else 0, xb)
        f, h = ffn_res(h, self.fc1, self.fc2, cfg.act, pact, rng.next_seed() if pact > 0 else 0)
        return norms.add_dropout_layer_norm(h, f, self.final_layer_norm.weight, self.final_layer_norm.bias, eps, p,
                                            rng.next_seed() if p > 0 else 0, xb)

    def forward_pre(self, normed, h, next_norm, mask=None, enc_out=None, enc_mask=None, cache=None, cross_kv=None):
        """Pre-LN layer (mBART / Pegasus) on (LN_self_attn(h), h) -> (next_norm(h'), h'): every residual update is
        fused with the LayerNorm that follows it (the next sub-layer's, or ``next_norm``: the next layer's first
        LayerNorm or the stack's final one)."""
        cfg = self.cfg
        tr = self.training
        p = cfg.dropout_rate if tr else 0.0
        pa = cfg.attention_dropout if tr else 0.0
        pact = cfg.activation_dropout if tr else 0.0
        eps = cfg.layer_norm_epsilon
        rng = default_rng()
        xb = _NORM_BIAS_COLSUM
        a = self.self_attn(normed, mask=None if self.is_decoder else mask, causal=self.is_decoder, p=pa, cache=cache)
        if self.is_decoder:
            normed, h = norms.add_dropout_layer_norm_pre(h, a, self.encoder_attn_layer_norm.weight,
                                                         self.encoder_attn_layer_norm.bias, eps, p,
                                                         rng.next_seed() if p > 0 else 0, xb)
            a = self.encoder_attn(normed, kv_in=enc_out, mask=enc_mask, p=pa, kv=cross_kv)
        normed, h = norms.add_dropout_layer_norm_pre(h, a, self.final_layer_norm.weight, self.final_layer_norm.bias,
                                                     eps, p, rng.next_seed() if p > 0 else 0, xb)
        f = ffn(normed, self.fc1, self.fc2, cfg.act, pact, rng.next_seed() if pact > 0 else 0)
        return norms.add_dropout_layer_norm_pre(h, f, next_norm.weight, next_norm.bias, eps, p,
                                                rng.next_seed() if p > 0 else 0, xb)


class BartLearnedPositionalEmbedding(nn.Embedding):
    offset = 2

    def __init__(self, n, d):
        super().__init__(n + self.offset, d)


class LearnedPositionalEmbedding0(BartLearnedPositionalEmbedding):
    """Blenderbot's learned positions: no offset (modeling_blenderbot.py BlenderbotLearnedPositionalEmbedding)."""
    offset = 0


class M2M100Positions(nn.Module):
    """Fixed positions of M2M100 / NLLB (modeling_m2m_100.py M2M100SinusoidalPositionalEmbedding): the tensor2tensor
    table [sin | cos] of t * 10000^(-i / (d/2 - 1)), row ``pad`` zero; a token's position is pad + 1 + (its index among
    the row's non-pad tokens, past cache length included), a pad token's is ``pad``.  Not in the checkpoint."""

    def __init__(self, n, d, pad):
        super().__init__()
        half = d // 2
        freq = torch.exp(torch.arange(half, dtype=torch.float32) * -(math.log(10000.0) / (half - 1)))
        ang = torch.arange(n + 2, dtype=torch.float32)[:, None] * freq[None, :]
        w = torch.cat([torch.sin(ang), torch.cos(ang)], dim=1)
        if d % 2 == 1:
            w = torch.cat([w, torch.zeros(n + 2, 1)], dim=1)
        w[pad] = 0.0
        self.pad = pad
        self.register_buffer("weight", w, persistent=False)

    def positions(self, input_ids, past: int):
        keep = input_ids.ne(self.pad).long()
        return (torch.cumsum(keep, dim=1) + past) * keep + self.pad


class SinusoidalPositions(nn.Module):
    """Fixed positions of Pegasus / Marian (modeling_pegasus.py PegasusSinusoidalPositionalEmbedding.create_weight):
    feature j of position t is sin / cos of t / 10000^(2 floor(j/2) / d), the sines in the first half of the features
    and the cosines in the second.  A persistent buffer named ``weight`` (the checkpoints carry it); never trained."""
    offset = 0
    derived_table = True  # models/hf_io.py: may be absent from a checkpoint (transformers' Marian does not save it)

    def __init__(self, n, d):
        super().__init__()
        pos = torch.arange(n, dtype=torch.float64)[:, None]
        j = torch.arange(d, dtype=torch.float64)[None, :]
        enc = pos / torch.pow(10000.0, 2 * torch.div(j, 2, rounding_mode="floor") / d)
        w = torch.empty(n, d, dtype=torch.float64)
        half = d // 2 if d % 2 == 0 else d // 2 + 1
        w[:, :half] = torch.sin(enc[:, 0::2])
        w[:, half:] = torch.cos(enc[:, 1::2])
        self.register_buffer("weight", w.float())


class BartStack(nn.Module):
    def __init__(self, cfg, is_decoder, embed_tokens):
        super().__init__()
        self.cfg = cfg
        self.is_decoder = is_decoder
        self._embed = [embed_tokens]
        if cfg.position_embedding == "sinusoidal_m2m":
            self.embed_positions = M2M100Positions(cfg.max_position_embeddings, cfg.d_model, cfg.pad_token_id)
            self._pos_offset = None
        else:
            pos_cls = {"sinusoidal": SinusoidalPositions, "learned0": LearnedPositionalEmbedding0}.get(
                cfg.position_embedding, BartLearnedPositionalEmbedding)
            self.embed_positions = pos_cls(cfg.max_position_embeddings, cfg.d_model)
            self._pos_offset = pos_cls.offset
        n = cfg.num_decoder_layers if is_decoder else cfg.num_layers
        self.layers = nn.ModuleList([BartLayer(cfg, is_decoder) for _ in range(n)])
        if cfg.layernorm_embedding:
            self.layernorm_embedding = nn.LayerNorm(cfg.d_model)
        if cfg.normalize_before:  # pre-LN stacks end with a LayerNorm (modeling_mbart.py MBartEncoder.layer_norm)
            self.layer_norm = nn.LayerNorm(cfg.d_model)
        self.embed_scale = math.sqrt(cfg.d_model) if cfg.scale_embedding else 1.0

    def cross_kv_linears(self):
        return [layer.encoder_attn.kv_proj for layer in self.layers]

    def project_cross_kv(self, enc_out):
        """All decoder layers' cross-attention K/V in ONE GEMM (ops/linear.py stacked_linear)."""
        B, S, _ = enc_out.shape
        H = self.cfg.num_heads
        return stacked_linear(enc_out, self.cross_kv_linears(), (B, S, 2, H, self.cfg.d_model // H))

    def forward(self, input_ids, attention_mask=None, enc_out=None, enc_mask=None, caches=None, q_offset=0,
                cross_kv=None):
        cfg = self.cfg
        p = cfg.dropout_rate if self.training else 0.0
        B, S = input_ids.shape
        x = embedding(input_ids, self._embed[0].weight, padding_idx=cfg.pad_token_id)
        if self.embed_scale != 1.0:
            x = x * self.embed_scale
        pw = self.embed_positions.weight
        if self._pos_offset is None:  # padding-aware positions, one row per sequence
            x = x + pw[self.embed_positions.positions(input_ids, q_offset)].to(x.dtype)
        else:
            pos = torch.arange(q_offset, q_offset + S, device=input_ids.device) + self._pos_offset
            x = x + (embedding(pos, pw) if pw.requires_grad else pw[pos].to(x.dtype)).unsqueeze(0)
        if cfg.layernorm_embedding:
            x = norms.layer_norm(x, self.layernorm_embedding.weight, self.layernorm_embedding.bias,
                                 cfg.layer_norm_epsilon)
        if self.is_decoder and cross_kv is None and enc_out is not None:
            cross_kv = self.project_cross_kv(enc_out)
        seed = default_rng().next_seed() if p > 0 else 0
        if cfg.normalize_before:
            return self._forward_pre(x, p, seed, attention_mask, enc_out, enc_mask, caches, cross_kv)
        h = activations.dropout(x, p, seed)
        for i, layer in enumerate(self.layers):
            cache = caches[i] if caches is not None else None
            ckv = cross_kv[i] if cross_kv is not None else None

            def run(h, layer=layer, cache=cache, ckv=ckv):
                return layer(h, mask=attention_mask, enc_out=enc_out, enc_mask=enc_mask, cache=cache, cross_kv=ckv)

            h = run_block(run, h, checkpoint=cfg.gradient_checkpointing and self.training and caches is None)
        return h

    def _forward_pre(self, x, p, seed, attention_mask, enc_out, enc_mask, caches, cross_kv):
        """Pre-LN stack: (LN_0(h), h) with h = dropout(embeddings), layer by layer, ending in (layer_norm(h), h)."""
        cfg = self.cfg
        layers = list(self.layers)
        normed, h = norms.dropout_layer_norm_pre(x, layers[0].self_attn_layer_norm.weight,
                                                 layers[0].self_attn_layer_norm.bias, cfg.layer_norm_epsilon, p, seed)
        for i, layer in enumerate(layers):
            nxt = layers[i + 1].self_attn_layer_norm if i + 1 < len(layers) else self.layer_norm
            cache = caches[i] if caches is not None else None
            ckv = cross_kv[i] if cross_kv is not None else None

            def run(normed, h, layer=layer, nxt=nxt, cache=cache, ckv=ckv):
                return layer.forward_pre(normed, h, nxt, mask=attention_mask, enc_out=enc_out, enc_mask=enc_mask,
                                         cache=cache, cross_kv=ckv)

            normed, h = run_block(run, normed, h, checkpoint=cfg.gradient_checkpointing and self.training and
                                  caches is None)
        return normed


class BartModel(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.shared = nn.Embedding(cfg.vocab_size, cfg.d_model, padding_idx=cfg.pad_token_id)
        self.encoder = BartStack(cfg, False, self.shared)
        self.decoder = BartStack(cfg, True, self.shared)


class BartForConditionalGeneration(nn.Module):
    """BART and the BART-family model types (``config.model_type`` bart / mbart / pegasus / marian)."""
    model_type = "bart"

    def __init__(self, cfg: Seq2SeqConfig):
        super().__init__()
        self.config = cfg
        self.model = BartModel(cfg)
        if cfg.final_logits_bias:  # BART / mBART / Pegasus / Marian; M2M100 has none
            self.register_buffer("final_logits_bias", torch.zeros(1, cfg.vocab_size))
        else:
            self.final_logits_bias = None
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        """PreTrainedModel._init_weights with init_std (Linear/Embedding ~ N(0, std), bias 0,
        padding row 0, LayerNorm 1/0) + final_logits_bias = 0 (modeling_bart.py:431-434)."""
        std = self.config.init_std
        for m in self.modules():
            if isinstance(m, nn.Linear):
                m.weight.normal_(0.0, std)
                if m.bias is not None:
                    m.bias.zero_()
            elif isinstance(m, nn.Embedding):
                m.weight.normal_(0.0, std)
                if m.padding_idx is not None:
                    m.weight[m.padding_idx].zero_()
            elif isinstance(m, nn.LayerNorm):
                m.weight.fill_(1.0)
                m.bias.zero_()
        if self.final_logits_bias is not None:
            self.final_logits_bias.zero_()

    def shift_right(self, labels):
        """shift_tokens_right (modeling_bart.py:58-71); mBART (modeling_mbart.py shift_tokens_right): the first
        decoder input is the label row's last non-pad token (the target language id) instead of a fixed id."""
        pad = self.config.pad_token_id
        if self.config.shift_mode == "mbart":
            prev = labels.masked_fill(labels == -100, pad)
            last = (prev.ne(pad).sum(dim=1) - 1).clamp(min=0).unsqueeze(-1)
            out = torch.empty_like(prev)
            out[:, 1:] = prev[:, :-1]
            out[:, 0] = prev.gather(1, last).squeeze(-1)
            return out
        out = labels.new_zeros(labels.shape)
        out[:, 1:] = labels[:, :-1]
        out[:, 0] = self.config.decoder_start_token_id
        out.masked_fill_(out == -100, pad)
        return out

    prepare_decoder_input_ids_from_labels = shift_right

    def encode(self, input_ids, attention_mask=None):
        return self.model.encoder(input_ids, attention_mask=attention_mask)

    def decode(self, decoder_input_ids, enc_out, enc_mask=None, caches=None, q_offset=0, cross_kv=None):
        return self.model.decoder(decoder_input_ids, enc_out=enc_out, enc_mask=enc_mask, caches=caches,
                                  q_offset=q_offset, cross_kv=cross_kv)

    def output_embedding(self):
        return self.model.shared.weight

    def logits_bias(self):
        return self.final_logits_bias.view(-1) if self.final_logits_bias is not None else None

    def lm_logits(self, hidden):
        logits = linear(hidden, self.output_embedding())
        return logits + self.final_logits_bias.to(hidden.dtype) if self.final_logits_bias is not None else logits

    def cross_attention_modules(self):
        return [layer.encoder_attn for layer in self.model.decoder.layers]

    def project_cross_kv(self, enc_out):
        return self.model.decoder.project_cross_kv(enc_out)

    def _dllm_param_groups(self):
        lin = self.model.decoder.cross_kv_linears()
        return [[m.weight for m in lin], [m.bias for m in lin]]

    def generate(self, input_ids, attention_mask=None, **kw):
        from .generation import generate
        return generate(self, input_ids, attention_mask=attention_mask, **kw)

    def enable_context_parallel(self, group=None, enable: bool = True):
        """BART is capped at 1024 learned positions (configuration_bart.py:50), so it has no long-sequence
        config to shard; context parallelism is implemented for the T5 family (models/t5.py)."""
        if enable:
            raise NotImplementedError("context parallelism is implemented for T5 / FLAN-T5 encoders only")
        return self

    def gradient_checkpointing_enable(self, enable: bool = True):
        """HF-style switch: recompute every layer in backward."""
        self.config.gradient_checkpointing = bool(enable)
        for st in (self.model.encoder, self.model.decoder):
            st.cfg = self.config
            for layer in st.layers:
                layer.cfg = self.config

    def forward(self, input_ids=None, attention_mask=None, decoder_input_ids=None, labels=None,
                label_smoothing: float = 0.0, return_logits: bool = False, encoder_outputs=None):
        enc = encoder_outputs if encoder_outputs is not None else self.encode(input_ids, attention_mask)
        if decoder_input_ids is None:
            decoder_input_ids = self.shift_right(labels)
        dec = self.decode(decoder_input_ids, enc, attention_mask)
        loss = None
        if labels is not None and not return_logits and wants_lm_head_loss(dec, labels.numel(), self.config.vocab_size):
            # LM head + CE with final_logits_bias, no materialised logits (ops/lm_head.py)
            loss = lm_head_loss(dec, self.output_embedding(), labels, bias=self.logits_bias(),
                                label_smoothing=label_smoothing)
            return Seq2SeqLMOutput(loss=loss, logits=None, encoder_last_hidden_state=enc)
        if labels is not None and not return_logits:
            raw = linear(dec, self.output_embedding())
            V = raw.shape[-1]
            loss = cross_entropy(raw.view(-1, V), labels.reshape(-1), bias=self.logits_bias(),
                                 label_smoothing=label_smoothing, inplace_grad=True)
            return Seq2SeqLMOutput(loss=loss, logits=None, encoder_last_hidden_state=enc)
        logits = self.lm_logits(dec)
        if labels is not None:
            V = logits.shape[-1]
            loss = cross_entropy(logits.view(-1, V), labels.reshape(-1), label_smoothing=label_smoothing)
        return Seq2SeqLMOutput(loss=loss, logits=logits, encoder_last_hidden_state=enc)
