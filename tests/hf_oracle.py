"""Build the transformers model that matches one of our configs and copy our weights into it."""
import torch

from distributed_llms_example_amd.models import to_hf_state_dict


def hf_model_for(model):
    import transformers
    cfg = model.config
    d = cfg.to_hf_dict()
    d.pop("architectures", None)
    d.pop("torch_dtype", None)
    mt = d.pop("model_type")
    classes = {"t5": (transformers.T5Config, transformers.T5ForConditionalGeneration),
               "mt5": (transformers.MT5Config, transformers.MT5ForConditionalGeneration),
               "umt5": (transformers.UMT5Config, transformers.UMT5ForConditionalGeneration),
               "bart": (transformers.BartConfig, transformers.BartForConditionalGeneration),
               "mbart": (transformers.MBartConfig, transformers.MBartForConditionalGeneration),
               "pegasus": (transformers.PegasusConfig, transformers.PegasusForConditionalGeneration),
               "marian": (transformers.MarianConfig, transformers.MarianMTModel),
               "m2m_100": (transformers.M2M100Config, transformers.M2M100ForConditionalGeneration),
               "plbart": (transformers.PLBartConfig, transformers.PLBartForConditionalGeneration),
               "blenderbot": (transformers.BlenderbotConfig, transformers.BlenderbotForConditionalGeneration)}
    cfg_cls, model_cls = classes[mt]
    # eager attention everywhere (the stacks' sub-configs included): transformers' SDPA path for UMT5 drops the
    # position bias and the decoder's causal mask
    hcfg = cfg_cls(**d, attn_implementation="eager")
    hf = model_cls(hcfg)
    sd = to_hf_state_dict(model)
    missing, unexpected = hf.load_state_dict(sd, strict=False)
    allowed = {"encoder.embed_tokens.weight", "decoder.embed_tokens.weight", "lm_head.weight",
               "model.encoder.embed_tokens.weight", "model.decoder.embed_tokens.weight"}
    bad = [m for m in missing if m not in allowed]
    assert not bad, bad
    assert not unexpected, unexpected
    return hf.to(dtype=next(model.parameters()).dtype)
