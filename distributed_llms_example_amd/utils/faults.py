"""Fault injection for recovery tests: kill or fail a rank at a chosen optimizer step.

    DLLM_FAULT_INJECT="step=5"                 every rank dies right after optimizer step 5
    DLLM_FAULT_INJECT="step=5,rank=1"          only rank 1 (the others then hit the process-group timeout /
                                               torchrun tears the group down, as with a real crash)
    DLLM_FAULT_INJECT="step=5,mode=raise"      raise InjectedFault instead of exiting (in-process tests)

``mode=exit`` (default) leaves with ``os._exit(43)``: no atexit handlers, no flushing of the process group,
like a worker killed by the OOM killer or a node fault.  Checkpoints written before the fault are what a
``--resume-from latest`` restart continues from.
"""
from __future__ import annotations

import os
import sys

EXIT_CODE = 43


class InjectedFault(RuntimeError):
    pass


def _spec():
    raw = os.environ.get("DLLM_FAULT_INJECT", "").strip()
    if not raw:
        return None
    kv = dict(item.split("=", 1) for item in raw.split(",") if "=" in item)
    return int(kv["step"]), (int(kv["rank"]) if "rank" in kv else None), kv.get("mode", "exit")


def maybe_inject(step: int, rank: int) -> None:
    spec = _spec()
    if spec is None:
        return
    at, who, mode = spec
    if step != at or (who is not None and who != rank):
        return
    msg = f"[fault-injection] rank {rank}: injected fault after step {step} (mode={mode})"
    print(msg, file=sys.stderr, flush=True)
    if mode == "raise":
        raise InjectedFault(msg)
    sys.stdout.flush()
    os._exit(EXIT_CODE)
