"""Tuned GEMM solution table for hipBLASLt / rocBLAS (PyTorch TunableOp), shipped in-tree.

The plain library GEMMs (projections, FFN, LM head) run on hipBLASLt/rocBLAS through torch.  Their
default heuristic picks are 5-30 % off the best solution for this model family's skinny-K shapes
(K = 768 / 1024 with 10^4-10^5 rows), so the best solution per (op, M, N, K) measured on MI355X is
recorded in ``configs/tunableop/<arch>.csv`` and replayed (tuning off) at start-up.  The CSV carries
validator lines (torch / HIP / hipBLASLt / rocBLAS versions, gfx arch); TunableOp ignores the table if
they do not match the running stack.  ``DLLM_TUNABLEOP=0`` disables; ``DLLM_TUNABLEOP=tune[:<dir>]`` re-tunes
unseen shapes and writes them to the per-process file (in <dir>; merge with tools/merge_tunableop.py).
"""
from __future__ import annotations

import os
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def enable(device_index: int = 0, arch: str = "gfx950") -> str | None:
    mode, _, tune_dir = os.environ.get("DLLM_TUNABLEOP", "1").partition(":")  # "tune:<dir>": results written there
    if mode == "0" or "PYTORCH_TUNABLEOP_ENABLED" in os.environ:
        return None
    # DLLM_TUNABLEOP_TABLE: another table (A/B of a re-tuned table against the shipped one)
    src = os.environ.get("DLLM_TUNABLEOP_TABLE") or os.path.join(ROOT, "configs", "tunableop", f"{arch}.csv")
    if not os.path.exists(src):
        return None
    d = tune_dir or tempfile.mkdtemp(prefix="dllm_tunableop_")
    os.makedirs(d, exist_ok=True)
    # every rank gets its own copy of the shared table (TunableOp may append to it)
    dst = os.path.join(d, f"tunableop_results{device_index}.csv")
    with open(src) as f, open(dst, "w") as g:
        g.write(f.read())
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "1"
    os.environ["PYTORCH_TUNABLEOP_TUNING"] = "1" if mode == "tune" else "0"
    os.environ["PYTORCH_TUNABLEOP_FILENAME"] = dst
    try:  # the env is read at first GEMM; set the same through the API and load the table now
        import torch.cuda.tunable as tunable
        tunable.enable(True)
        tunable.tuning_enable(mode == "tune")
        tunable.set_filename(dst, insert_device_ordinal=False)
        tunable.read_file(dst)
    except Exception:
        pass
    return dst
