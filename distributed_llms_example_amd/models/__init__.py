"""Encoder-decoder model families on the fused-op library: T5 / mT5 / FLAN-T5 (models/t5.py) and BART / mBART /
Pegasus / Marian / M2M100-NLLB / PLBart /
Blenderbot (models/bart.py)."""
from .bart import BartForConditionalGeneration
from .config import PRESETS, Seq2SeqConfig, resolve_config
from .hf_io import build_model, from_hf_state_dict, from_pretrained, save_pretrained, to_hf_state_dict
from .t5 import T5ForConditionalGeneration

__all__ = ["PRESETS", "Seq2SeqConfig", "resolve_config", "build_model", "from_pretrained", "save_pretrained",
           "to_hf_state_dict", "from_hf_state_dict", "T5ForConditionalGeneration", "BartForConditionalGeneration"]
