"""Shared command-line surface of the three entry points.

The six flags of the reference are kept verbatim (ref/train-torchrun.py:183-188,
ref/train-accelerator.py:320-325, ref/train-task.py:411-416); everything else is optional and
defaults to reference semantics.  Data comes from the Valohai ``dataset``
input (``train.json``/``val.json``), or ``--data-dir``, or ``--synthetic N`` (offline runs).
"""
from __future__ import annotations

import argparse
import os

from .data.dataset import convert_examples_to_features, load_samsum, synthetic_samsum_records
from .data.tokenization import load_tokenizer
from .models.config import resolve_config
from .ops import routing
from .platform import valohai


def bucket_mb_arg(v: str):
    """``--bucket-mb``: a size in MiB or ``auto``."""
    return "auto" if str(v).lower() == "auto" else float(v)


def base_parser(description: str, defaults: dict | None = None) -> argparse.ArgumentParser:
    d = {"batch_size": 1, "num_epochs": 1, "warmup_steps": 500, "evaluation_steps": 500}
    d.update(defaults or {})
    ap = argparse.ArgumentParser(description=description)
    ap.add_argument("--model-ckpt", type=str, default="facebook/bart-large-cnn", help="Pretrained model checkpoint")
    ap.add_argument("--output-dir", type=str, default="bart-large-cnn", help="Output directory for the trained model")
    ap.add_argument("--batch-size", type=int, default=d["batch_size"], help="Batch size")
    ap.add_argument("--num-epochs", type=int, default=d["num_epochs"], help="Number of training epochs")
    ap.add_argument("--warmup-steps", type=int, default=d["warmup_steps"], help="Warmup steps")
    ap.add_argument("--evaluation-steps", type=int, default=d["evaluation_steps"], help="Evaluation steps")
    g = ap.add_argument_group("MI355X framework options (defaults reproduce the reference)")
    g.add_argument("--data-dir", type=str, default=None, help="directory with train.json/val.json")
    g.add_argument("--synthetic", type=int, default=0, help="use N synthetic SAMSum-schema records")
    g.add_argument("--max-source-length", type=int, default=1024)
    g.add_argument("--max-target-length", type=int, default=128)
    g.add_argument("--ignore-pad-labels", action="store_true", help="mask pad tokens out of the loss")
    g.add_argument("--precision", choices=["bf16", "fp32"], default=None, help="default: bf16 on GPU, fp32 on CPU")
    g.add_argument("--grad-accum", type=int, default=None)
    g.add_argument("--coalesce-grad-accum", type=str, default="auto",
                   help="run gradient-accumulation micro-batches as fewer larger passes: 'auto' (as many as the "
                        "first step's measured activation memory allows in 60%% of HBM), N (max samples per pass), 0 off")
    g.add_argument("--learning-rate", type=float, default=5e-5)
    g.add_argument("--max-steps", type=int, default=-1)
    g.add_argument("--bucket-mb", type=bucket_mb_arg, default="auto",
                   help="gradient all-reduce bucket size in MiB, or 'auto' (default: probe RCCL's bus bandwidth over "
                        "32-256 MiB on the job's process group and take the smallest size within 5%% of the best)")
    g.add_argument("--no-overlap", action="store_true",
                   help="all-reduce after backward instead of overlapping (HIP-graph steps: the post-backward "
                        "'split' schedule)")
    g.add_argument("--grad-reduce-dtype", choices=["fp32", "bf16"], default="fp32",
                   help="dtype of the gradient all-reduce on the wire: bf16 halves the xGMI bytes; gradients are still "
                        "accumulated in fp32 and widened back after each bucket's all-reduce")
    g.add_argument("--eval-batch-size", type=int, default=None)
    g.add_argument("--max-eval-samples", type=int, default=None)
    g.add_argument("--gen-max-length", type=int, default=128)
    g.add_argument("--num-beams", type=int, default=2)
    g.add_argument("--resume-from", type=str, default=None, help="checkpoint dir, or 'latest'")
    g.add_argument("--save-steps", type=int, default=None,
                   help="full training checkpoint every N optimizer steps (reference: final only)")
    g.add_argument("--seed", type=int, default=42)
    g.add_argument("--gradient-checkpointing", action="store_true",
                   help="recompute each transformer block in backward (long sequences / large models)")
    g.add_argument("--context-parallel", type=int, default=1,
                   help="shard the encoder sequence over groups of N ranks (ring attention; T5 family)")
    g.add_argument("--model-overrides", type=str, default=None,
                   help="comma list key=value applied to the model config (e.g. num_layers=2)")
    return ap


# Evaluation / generation batch when --eval-batch-size is not given.  Beam-search generation is launch-bound at small
# batches (t5-base, 818 samples, num_beams=2, one MI355X: 107 samples/s at batch 64, 195 at 128, 299 at 256, 480 with
# all 818 at once; tools/eval_bench.py, profiles/r2_eval_batch.txt), and a 288 GB GPU holds the caches of hundreds of
# sequences, so GPU runs evaluate in batches of at least this many samples (the reference evaluates with its training
# batch size, or 1 in train-accelerator).  Results are the same per sample.
def gpu_eval_batch() -> int:
    return int(routing.get("eval_batch"))


def eval_batch_size(args, device) -> int:
    if getattr(args, "eval_batch_size", None):
        return args.eval_batch_size
    bs = args.batch_size or 1
    return max(bs, gpu_eval_batch()) if getattr(device, "type", str(device)) == "cuda" else bs


def apply_overrides(cfg, spec: str | None):
    if not spec:
        return cfg
    kv = {}
    for item in spec.split(","):
        k, v = item.split("=")
        cur = getattr(cfg, k)
        kv[k] = type(cur)(v) if not isinstance(cur, bool) else v.lower() in ("1", "true", "yes")
    if "num_layers" in kv and "num_decoder_layers" not in kv:
        kv["num_decoder_layers"] = kv["num_layers"]
    return cfg.replace(**kv)


def load_records(args):
    if args.synthetic:
        n = args.synthetic
        return {"train": synthetic_samsum_records(n, args.seed), "validation": synthetic_samsum_records(max(4, n // 4),
                                                                                                    args.seed + 1)}
    data_dir = args.data_dir or os.path.dirname(valohai.inputs("dataset").path())
    return load_samsum(data_dir)


def build_data(args, cfg):
    """(tokenizer, train_features, eval_features, eval_records) following convert_examples_to_features."""
    recs = load_records(args)
    tok = load_tokenizer(args.model_ckpt, cfg, texts=[r["dialogue"] for r in recs["train"]] +
                         [r["summary"] for r in recs["train"]])
    tr = convert_examples_to_features(recs["train"], tok, args.max_source_length, args.max_target_length,
                                      ignore_pad_labels=args.ignore_pad_labels)
    ev_recs = recs["validation"][: args.max_eval_samples] if args.max_eval_samples else recs["validation"]
    ev = convert_examples_to_features(ev_recs, tok, args.max_source_length, args.max_target_length,
                                      ignore_pad_labels=args.ignore_pad_labels)
    return tok, tr, ev


def model_config(args):
    cfg = apply_overrides(resolve_config(args.model_ckpt), args.model_overrides)
    if getattr(args, "gradient_checkpointing", False):
        cfg = cfg.replace(gradient_checkpointing=True)
    return cfg
