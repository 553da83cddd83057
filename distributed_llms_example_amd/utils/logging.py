"""Rank-gated logging and JSON-line metrics.

The reference's observability is stdout JSON lines that Valohai ingests as execution metadata
(``PrinterCallback`` ref/train-torchrun.py:144-147; ``dump_valohai_metadata`` ref/train-accelerator.py:283)
plus Python logging at INFO on the local main process and ERROR elsewhere (``set_logs``,
ref/train-accelerator.py:45-51).  Same keys here; only the main process prints metrics.
"""
from __future__ import annotations

import json
import logging
import math
import sys


def get_logger(name: str = "distributed_llms_example_amd") -> logging.Logger:
    return logging.getLogger(name)


def setup_logging(is_local_main: bool, level=logging.INFO):
    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(name)s - %(message)s", datefmt="%m/%d/%Y %H:%M:%S",
                        stream=sys.stderr)
    get_logger().setLevel(level if is_local_main else logging.ERROR)


def _clean(v):
    if hasattr(v, "item"):
        v = v.item()
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return str(v)
    return v


def dump_metrics(logs: dict, is_main: bool = True, stream=None):
    """Print one JSON line (Valohai metadata)."""
    if not is_main:
        return
    logs = {k: _clean(v) for k, v in logs.items() if k != "total_flos"}
    print(json.dumps(logs), file=stream or sys.stdout, flush=True)
