"""Model configurations for the seq2seq families the reference fine-tunes.

The reference loads every model through ``AutoModelForSeq2SeqLM.from_pretrained(model_ckpt)``
(ref/train-torchrun.py:35, ref/train-accelerator.py:41, ref/train-task.py:83); the default
checkpoint is ``facebook/bart-large-cnn`` (ref/valohai.yaml:10,36,65) and the benchmark family is
T5 (BASELINE.json).  There is no network here, so the public configs are encoded as presets and
weights are random-initialised with the HF initialisation rules (SURVEY.md §7.3 "Offline
environment").  ``Seq2SeqConfig.to_hf_dict`` / ``from_hf_dict`` read and write an HF
``config.json`` so checkpoints round-trip with ``transformers``.
"""
from __future__ import annotations

import copy
import dataclasses
import json
import os
from dataclasses import dataclass, field


@dataclass
class Seq2SeqConfig:
    model_type: str = "t5"  # "t5" | BART family: "bart" | "mbart" | "pegasus" | "marian" | "m2m_100" | "plbart" | "blenderbot"
    # T5 implementation variants: "t5" / "mt5" (same layers), "umt5" (every self-attention layer owns its
    # relative-position bias table: modeling_umt5.py UMT5LayerSelfAttention, has_relative_attention_bias=True)
    t5_flavor: str = "t5"
    vocab_size: int = 32128
    d_model: int = 512
    d_kv: int = 64
    d_ff: int = 2048
    num_layers: int = 6
    num_decoder_layers: int = 6
    num_heads: int = 8
    # T5 relative position bias (modeling_t5.py:217-279)
    relative_attention_num_buckets: int = 32
    relative_attention_max_distance: int = 128
    # "relu" (T5 v1.0), "gated-gelu" (flan / v1.1, gelu_new), "gelu" (BART, erf)
    feed_forward_proj: str = "relu"
    dropout_rate: float = 0.1
    attention_dropout: float = 0.1  # T5 applies dropout_rate to probs; BART uses attention_dropout
    activation_dropout: float = 0.0  # BART only (T5 uses dropout_rate inside the FFN)
    layer_norm_epsilon: float = 1e-6
    initializer_factor: float = 1.0  # T5
    init_std: float = 0.02  # BART
    tie_word_embeddings: bool = True
    # recompute each transformer block in backward (O(layers) less activation memory; long sequences)
    gradient_checkpointing: bool = False
    scale_decoder_outputs: bool = True  # T5: scale by d_model**-0.5 before lm_head when tied
    # BART specifics
    max_position_embeddings: int = 1024
    scale_embedding: bool = False
    final_logits_bias: bool = False
    # BART-family variants (transformers modeling_mbart.py / modeling_pegasus.py / modeling_marian.py):
    # pre-LN layers with a final LayerNorm per stack (mBART, Pegasus) vs post-LN (BART, Marian); LayerNorm after
    # the embeddings (BART, mBART); learned positions with offset 2 (BART, mBART) vs fixed sinusoidal (Pegasus,
    # Marian); decoder start token = the last non-pad label token (mBART's language id) vs a fixed id
    normalize_before: bool = False
    layernorm_embedding: bool = True
    position_embedding: str = "learned"  # "learned" (offset 2) | "learned0" | "sinusoidal" | "sinusoidal_m2m"
    shift_mode: str = "standard"  # "standard" | "mbart"
    # special tokens
    pad_token_id: int = 0
    eos_token_id: int = 1
    bos_token_id: int | None = None
    decoder_start_token_id: int = 0
    forced_bos_token_id: int | None = None
    forced_eos_token_id: int | None = None
    # generation defaults written to generation_config.json
    generation: dict = field(default_factory=dict)
    name: str = ""

    @property
    def inner_dim(self) -> int:
        return self.num_heads * self.d_kv

    @property
    def is_gated(self) -> bool:
        return self.feed_forward_proj.startswith("gated")

    @property
    def per_layer_position_bias(self) -> bool:
        return self.model_type == "t5" and self.t5_flavor == "umt5"

    @property
    def act(self) -> str:
        a = self.feed_forward_proj.split("-")[-1]
        if self.feed_forward_proj == "gated-gelu":
            return "gelu_new"
        if a == "swish":  # Marian's name for SiLU
            return "silu"
        return a

    def replace(self, **kw) -> "Seq2SeqConfig":
        c = copy.deepcopy(self)
        for k, v in kw.items():
            if not hasattr(c, k):
                raise AttributeError(k)
            setattr(c, k, v)
        return c

    # ---------------------------------------------------------------- HF config.json I/O
    def to_hf_dict(self) -> dict:
        if self.model_type == "t5":
            d = {
                "architectures": [{"t5": "T5ForConditionalGeneration", "mt5": "MT5ForConditionalGeneration",
                                   "umt5": "UMT5ForConditionalGeneration"}[self.t5_flavor]],
                "model_type": self.t5_flavor,
                "vocab_size": self.vocab_size,
                "d_model": self.d_model,
                "d_kv": self.d_kv,
                "d_ff": self.d_ff,
                "num_layers": self.num_layers,
                "num_decoder_layers": self.num_decoder_layers,
                "num_heads": self.num_heads,
                "relative_attention_num_buckets": self.relative_attention_num_buckets,
                "relative_attention_max_distance": self.relative_attention_max_distance,
                "dropout_rate": self.dropout_rate,
                "layer_norm_epsilon": self.layer_norm_epsilon,
                "initializer_factor": self.initializer_factor,
                "feed_forward_proj": self.feed_forward_proj,
                "is_encoder_decoder": True,
                "pad_token_id": self.pad_token_id,
                "eos_token_id": self.eos_token_id,
                "decoder_start_token_id": self.decoder_start_token_id,
                "tie_word_embeddings": self.tie_word_embeddings,
            }
        else:
            arch = {"bart": "BartForConditionalGeneration", "mbart": "MBartForConditionalGeneration",
                    "pegasus": "PegasusForConditionalGeneration", "marian": "MarianMTModel",
                    "m2m_100": "M2M100ForConditionalGeneration", "plbart": "PLBartForConditionalGeneration",
                    "blenderbot": "BlenderbotForConditionalGeneration"}[self.model_type]
            d = {
                "architectures": [arch],
                "model_type": self.model_type,
                "vocab_size": self.vocab_size,
                "d_model": self.d_model,
                "encoder_layers": self.num_layers,
                "decoder_layers": self.num_decoder_layers,
                "encoder_attention_heads": self.num_heads,
                "decoder_attention_heads": self.num_heads,
                "encoder_ffn_dim": self.d_ff,
                "decoder_ffn_dim": self.d_ff,
                "activation_function": self.feed_forward_proj,
                "dropout": self.dropout_rate,
                "attention_dropout": self.attention_dropout,
                "activation_dropout": self.activation_dropout,
                "init_std": self.init_std,
                "max_position_embeddings": self.max_position_embeddings,
                "scale_embedding": self.scale_embedding,
                "is_encoder_decoder": True,
                "pad_token_id": self.pad_token_id,
                "bos_token_id": self.bos_token_id,
                "eos_token_id": self.eos_token_id,
                "decoder_start_token_id": self.decoder_start_token_id,
                "forced_bos_token_id": self.forced_bos_token_id,
                "forced_eos_token_id": self.forced_eos_token_id,
                "tie_word_embeddings": True,
                "encoder_layerdrop": 0.0,
                "decoder_layerdrop": 0.0,
            }
            if self.model_type == "marian":
                d["decoder_vocab_size"] = self.vocab_size
                d["share_encoder_decoder_embeddings"] = True
        d["torch_dtype"] = "float32"
        return d

    @classmethod
    def from_hf_dict(cls, d: dict) -> "Seq2SeqConfig":
        mt = d.get("model_type", "t5")
        if mt in ("t5", "mt5", "umt5"):
            ff = d.get("feed_forward_proj", "relu")
            nl = d.get("num_layers", 6)
            tie = d.get("tie_word_embeddings", True)
            return cls(
                model_type="t5", t5_flavor=mt, vocab_size=d.get("vocab_size", 32128), d_model=d.get("d_model", 512),
                d_kv=d.get("d_kv", 64), d_ff=d.get("d_ff", 2048), num_layers=nl,
                num_decoder_layers=d.get("num_decoder_layers") or nl, num_heads=d.get("num_heads", 8),
                relative_attention_num_buckets=d.get("relative_attention_num_buckets", 32),
                relative_attention_max_distance=d.get("relative_attention_max_distance", 128),
                feed_forward_proj=ff, dropout_rate=d.get("dropout_rate", 0.1),
                attention_dropout=d.get("dropout_rate", 0.1),
                layer_norm_epsilon=d.get("layer_norm_epsilon", 1e-6),
                initializer_factor=d.get("initializer_factor", 1.0),
                tie_word_embeddings=tie, scale_decoder_outputs=tie,
                pad_token_id=d.get("pad_token_id", 0), eos_token_id=_first(d.get("eos_token_id", 1)),
                decoder_start_token_id=d.get("decoder_start_token_id", 0) or 0,
            )
        if mt in _FAMILY:
            fam = {"final_logits_bias": True, **_FAMILY[mt]}
            return cls(
                model_type=mt, vocab_size=d.get("vocab_size", 50265), d_model=d.get("d_model", 1024),
                d_kv=d.get("d_model", 1024) // d.get("encoder_attention_heads", 16),
                d_ff=d.get("encoder_ffn_dim", 4096), num_layers=d.get("encoder_layers", 12),
                num_decoder_layers=d.get("decoder_layers", 12), num_heads=d.get("encoder_attention_heads", 16),
                feed_forward_proj=d.get("activation_function", "gelu"), dropout_rate=d.get("dropout", 0.1),
                attention_dropout=d.get("attention_dropout", 0.0),
                activation_dropout=d.get("activation_dropout", 0.0), layer_norm_epsilon=1e-5,
                init_std=d.get("init_std", 0.02), max_position_embeddings=d.get("max_position_embeddings", 1024),
                scale_embedding=d.get("scale_embedding", False),
                tie_word_embeddings=True, scale_decoder_outputs=False,
                pad_token_id=d.get("pad_token_id", 1), eos_token_id=_first(d.get("eos_token_id", 2)),
                bos_token_id=d.get("bos_token_id", 0 if mt in ("bart", "mbart") else None),
                decoder_start_token_id=d.get("decoder_start_token_id") if d.get("decoder_start_token_id") is not None
                else (d.get("pad_token_id", 1) if mt != "bart" else 2),
                forced_bos_token_id=d.get("forced_bos_token_id"), forced_eos_token_id=d.get("forced_eos_token_id", 2),
                **fam,
            )
        raise ValueError(f"unsupported model_type {mt!r}")

    def save(self, path: str) -> None:
        with open(os.path.join(path, "config.json"), "w") as f:
            json.dump(self.to_hf_dict(), f, indent=2, sort_keys=True)
        with open(os.path.join(path, "generation_config.json"), "w") as f:
            json.dump(self.generation_config_dict(), f, indent=2, sort_keys=True)

    def generation_config_dict(self) -> dict:
        g = {"decoder_start_token_id": self.decoder_start_token_id, "eos_token_id": self.eos_token_id,
             "pad_token_id": self.pad_token_id}
        if self.bos_token_id is not None:
            g["bos_token_id"] = self.bos_token_id
        if self.forced_bos_token_id is not None:
            g["forced_bos_token_id"] = self.forced_bos_token_id
        if self.forced_eos_token_id is not None:
            g["forced_eos_token_id"] = self.forced_eos_token_id
        g.update(self.generation)
        return g

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


def _first(x):
    return x[0] if isinstance(x, (list, tuple)) else x


# structural switches of the BART-family model types (see the Seq2SeqConfig fields)
_FAMILY = {
    "bart": dict(normalize_before=False, layernorm_embedding=True, position_embedding="learned", shift_mode="standard"),
    "mbart": dict(normalize_before=True, layernorm_embedding=True, position_embedding="learned", shift_mode="mbart"),
    "pegasus": dict(normalize_before=True, layernorm_embedding=False, position_embedding="sinusoidal",
                    shift_mode="standard"),
    "marian": dict(normalize_before=False, layernorm_embedding=False, position_embedding="sinusoidal",
                   shift_mode="standard"),
    # PLBart: BART layers with mBART's language-id decoder start (modeling_plbart.py)
    "plbart": dict(normalize_before=False, layernorm_embedding=True, position_embedding="learned", shift_mode="mbart"),
    # Blenderbot: pre-LN, learned positions without offset, no embedding LayerNorm (modeling_blenderbot.py)
    "blenderbot": dict(normalize_before=True, layernorm_embedding=False, position_embedding="learned0",
                       shift_mode="standard"),
    # M2M100 / NLLB: pre-LN, padding-aware sinusoidal positions (modeling_m2m_100.py), no final_logits_bias
    "m2m_100": dict(normalize_before=True, layernorm_embedding=False, position_embedding="sinusoidal_m2m",
                    shift_mode="standard", final_logits_bias=False),
}


def _bartlike(mt, name, vocab, d_model, layers, heads, d_ff, act, max_pos, scale_emb, pad, eos, bos, start,
              dropout=0.1, attn_dropout=0.0, act_dropout=0.0, forced_bos=None, forced_eos=None, dec_layers=None):
    return Seq2SeqConfig(
        model_type=mt, name=name, vocab_size=vocab, d_model=d_model, d_kv=d_model // heads, d_ff=d_ff,
        num_layers=layers, num_decoder_layers=dec_layers or layers, num_heads=heads, feed_forward_proj=act, dropout_rate=dropout,
        attention_dropout=attn_dropout, activation_dropout=act_dropout, layer_norm_epsilon=1e-5,
        scale_decoder_outputs=False, max_position_embeddings=max_pos,
        scale_embedding=scale_emb, pad_token_id=pad, eos_token_id=eos, bos_token_id=bos, decoder_start_token_id=start,
        forced_bos_token_id=forced_bos, forced_eos_token_id=forced_eos, **{"final_logits_bias": True, **_FAMILY[mt]})


def _t5(name, d_model, d_ff, layers, heads, ff="relu", tie=True, vocab=32128, d_kv=64, flavor="t5"):
    return Seq2SeqConfig(model_type="t5", t5_flavor=flavor, name=name, vocab_size=vocab, d_model=d_model, d_kv=d_kv,
                         d_ff=d_ff,
                         num_layers=layers, num_decoder_layers=layers, num_heads=heads, feed_forward_proj=ff,
                         tie_word_embeddings=tie, scale_decoder_outputs=tie)


# Public architecture hyper-parameters (SURVEY.md §2.4 "Model sizes").
PRESETS: dict[str, Seq2SeqConfig] = {
    "t5-small": _t5("t5-small", 512, 2048, 6, 8),
    "t5-base": _t5("t5-base", 768, 3072, 12, 12),
    "t5-large": _t5("t5-large", 1024, 4096, 24, 16),
    "flan-t5-small": _t5("flan-t5-small", 512, 1024, 8, 6, ff="gated-gelu", tie=False),
    "flan-t5-base": _t5("flan-t5-base", 768, 2048, 12, 12, ff="gated-gelu", tie=False),
    "flan-t5-large": _t5("flan-t5-large", 1024, 2816, 24, 16, ff="gated-gelu", tie=False),
    "flan-t5-xl": _t5("flan-t5-xl", 2048, 5120, 24, 32, ff="gated-gelu", tie=False),
    # T5 v1.1 and mT5 (multilingual: 250K SentencePiece vocabulary): the FLAN-T5 architecture
    "t5-v1_1-base": _t5("t5-v1_1-base", 768, 2048, 12, 12, ff="gated-gelu", tie=False),
    "t5-v1_1-large": _t5("t5-v1_1-large", 1024, 2816, 24, 16, ff="gated-gelu", tie=False),
    "mt5-small": _t5("mt5-small", 512, 1024, 8, 6, ff="gated-gelu", tie=False, vocab=250112, flavor="mt5"),
    "mt5-base": _t5("mt5-base", 768, 2048, 12, 12, ff="gated-gelu", tie=False, vocab=250112, flavor="mt5"),
    "mt5-large": _t5("mt5-large", 1024, 2816, 24, 16, ff="gated-gelu", tie=False, vocab=250112, flavor="mt5"),
    # UMT5: the mT5 architecture with a relative-position bias table in every self-attention layer
    "umt5-small": _t5("umt5-small", 512, 1024, 8, 6, ff="gated-gelu", tie=False, vocab=256384, flavor="umt5"),
    "umt5-base": _t5("umt5-base", 768, 2048, 12, 12, ff="gated-gelu", tie=False, vocab=256384, flavor="umt5"),
    "umt5-xl": _t5("umt5-xl", 2048, 5120, 24, 32, ff="gated-gelu", tie=False, vocab=256384, flavor="umt5"),
    "bart-base": Seq2SeqConfig(
        model_type="bart", name="bart-base", vocab_size=50265, d_model=768, d_kv=64, d_ff=3072, num_layers=6,
        num_decoder_layers=6, num_heads=12, feed_forward_proj="gelu", dropout_rate=0.1, attention_dropout=0.0,
        activation_dropout=0.0, layer_norm_epsilon=1e-5, final_logits_bias=True, scale_decoder_outputs=False,
        pad_token_id=1, eos_token_id=2, bos_token_id=0, decoder_start_token_id=2, forced_bos_token_id=0,
        forced_eos_token_id=2),
    "bart-large": Seq2SeqConfig(
        model_type="bart", name="bart-large", vocab_size=50265, d_model=1024, d_kv=64, d_ff=4096, num_layers=12,
        num_decoder_layers=12, num_heads=16, feed_forward_proj="gelu", dropout_rate=0.1, attention_dropout=0.0,
        activation_dropout=0.0, layer_norm_epsilon=1e-5, final_logits_bias=True, scale_decoder_outputs=False,
        pad_token_id=1, eos_token_id=2, bos_token_id=0, decoder_start_token_id=2, forced_bos_token_id=0,
        forced_eos_token_id=2),
}
# bart-large-cnn: vocab 50264 and CNN/DM generation defaults.
PRESETS["bart-large-cnn"] = PRESETS["bart-large"].replace(
    name="bart-large-cnn", vocab_size=50264,
    generation={"min_length": 56, "max_length": 142, "length_penalty": 2.0, "no_repeat_ngram_size": 3,
                "num_beams": 4, "early_stopping": True})
# other AutoModelForSeq2SeqLM families on the BART implementation (models/bart.py; public config.json values)
PRESETS["mbart-large-cc25"] = _bartlike("mbart", "mbart-large-cc25", 250027, 1024, 12, 16, 4096, "gelu", 1024, True,
                                        pad=1, eos=2, bos=0, start=2, forced_eos=2)
PRESETS["mbart-large-50"] = PRESETS["mbart-large-cc25"].replace(name="mbart-large-50", vocab_size=250054)
PRESETS["pegasus-large"] = _bartlike("pegasus", "pegasus-large", 96103, 1024, 16, 16, 4096, "relu", 1024, True,
                                     pad=0, eos=1, bos=None, start=0, attn_dropout=0.1, act_dropout=0.1, forced_eos=1)
PRESETS["pegasus-xsum"] = PRESETS["pegasus-large"].replace(
    name="pegasus-xsum", max_position_embeddings=512,
    generation={"max_length": 64, "length_penalty": 0.6, "num_beams": 8})
PRESETS["opus-mt-en-de"] = _bartlike("marian", "opus-mt-en-de", 58101, 512, 6, 8, 2048, "swish", 512, True,
                                     pad=58100, eos=0, bos=None, start=58100, forced_eos=0)
PRESETS["m2m100_418m"] = _bartlike("m2m_100", "m2m100_418m", 128112, 1024, 12, 16, 4096, "relu", 1024, True,
                                   pad=1, eos=2, bos=0, start=2, attn_dropout=0.1, forced_eos=2)
PRESETS["plbart-base"] = _bartlike("plbart", "plbart-base", 50005, 768, 6, 12, 3072, "gelu", 1024, True, pad=1, eos=2,
                                   bos=0, start=2, forced_eos=2)
PRESETS["blenderbot-400m-distill"] = _bartlike("blenderbot", "blenderbot-400m-distill", 8008, 1280, 2, 32, 5120,
                                               "gelu", 128, True, pad=0, eos=2, bos=1, start=1, forced_eos=2,
                                               dec_layers=12)
PRESETS["nllb-200-distilled-600m"] = PRESETS["m2m100_418m"].replace(name="nllb-200-distilled-600m", vocab_size=256206)
# tiny configs for CPU tests
PRESETS["t5-tiny"] = _t5("t5-tiny", 64, 128, 2, 4, vocab=512, d_kv=16)
PRESETS["t5-tiny-gated"] = _t5("t5-tiny-gated", 64, 96, 2, 4, ff="gated-gelu", tie=False, vocab=512, d_kv=16)
PRESETS["umt5-tiny"] = _t5("umt5-tiny", 64, 96, 2, 4, ff="gated-gelu", tie=True, vocab=512, d_kv=16, flavor="umt5")
PRESETS["bart-tiny"] = PRESETS["bart-base"].replace(name="bart-tiny", vocab_size=512, d_model=64, d_kv=16, d_ff=128,
                                                    num_layers=2, num_decoder_layers=2, num_heads=4,
                                                    max_position_embeddings=256)
PRESETS["mbart-tiny"] = _bartlike("mbart", "mbart-tiny", 512, 64, 2, 4, 128, "gelu", 256, True, pad=1, eos=2, bos=0,
                                  start=2, forced_eos=2)
PRESETS["pegasus-tiny"] = _bartlike("pegasus", "pegasus-tiny", 512, 64, 2, 4, 128, "relu", 256, True, pad=0, eos=1,
                                    bos=None, start=0, attn_dropout=0.1, act_dropout=0.1, forced_eos=1)
PRESETS["m2m100-tiny"] = _bartlike("m2m_100", "m2m100-tiny", 512, 64, 2, 4, 128, "relu", 256, True, pad=1, eos=2,
                                   bos=0, start=2, attn_dropout=0.1, forced_eos=2)
PRESETS["plbart-tiny"] = _bartlike("plbart", "plbart-tiny", 512, 64, 2, 4, 128, "gelu", 256, True, pad=1, eos=2, bos=0,
                                   start=2, forced_eos=2)
PRESETS["blenderbot-tiny"] = _bartlike("blenderbot", "blenderbot-tiny", 512, 64, 1, 4, 128, "gelu", 256, True, pad=0,
                                       eos=2, bos=1, start=1, forced_eos=2, dec_layers=2)
PRESETS["marian-tiny"] = _bartlike("marian", "marian-tiny", 512, 64, 2, 4, 128, "swish", 256, True, pad=511, eos=0,
                                   bos=None, start=511, forced_eos=0)


def resolve_config(name_or_path: str) -> Seq2SeqConfig:
    """Map an HF checkpoint id (``google-t5/t5-base``, ``facebook/bart-large-cnn``) or a local
    directory with ``config.json`` to a config."""
    if name_or_path and os.path.isdir(name_or_path) and os.path.exists(os.path.join(name_or_path, "config.json")):
        with open(os.path.join(name_or_path, "config.json")) as f:
            cfg = Seq2SeqConfig.from_hf_dict(json.load(f))
        cfg.name = name_or_path
        gpath = os.path.join(name_or_path, "generation_config.json")
        if os.path.exists(gpath):
            with open(gpath) as f:
                g = json.load(f)
            keep = {"min_length", "max_length", "length_penalty", "no_repeat_ngram_size", "num_beams",
                    "early_stopping"}
            cfg.generation = {k: v for k, v in g.items() if k in keep}
        return cfg
    key = (name_or_path or "t5-small").split("/")[-1].lower()
    if key not in PRESETS:
        raise KeyError(f"unknown model {name_or_path!r}; presets: {sorted(PRESETS)}")
    return copy.deepcopy(PRESETS[key])
