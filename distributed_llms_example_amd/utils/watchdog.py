"""Per-step stall watchdog for multi-rank runs.

A rank whose collective partner never arrives does not fail: its RCCL kernel spins and the host keeps queueing work
until the next synchronisation point blocks — and ProcessGroupNCCL's own watchdog only fires after the process-group
timeout (30 min by default), with a message that does not say where in the step the rank stood.  ``StepWatchdog``
bounds a step instead: every step is bracketed (``begin`` / ``end``; on the GPU ``end`` records an event that the
watchdog thread polls, so no host synchronisation is added), and a step not finished ``timeout_s`` seconds after it
began makes the thread print the rank, the step, and what the caller's ``describe`` reports (the reducer's launch
cursor: which bucket all-reduces of the step were issued), then end the process with exit status 3 — no re-exec, no
retry: the launcher (torchrun / Valohai) sees a failed rank and tears the job down.

``DLLM_STEP_TIMEOUT`` (seconds, default 1800; 0 disables) sets the bound; the first steps (graph capture, kernel
tables) must fit in it.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from collections import deque

import torch

EXIT_STALL = 3


def default_timeout() -> float:
    return float(os.environ.get("DLLM_STEP_TIMEOUT", "1800"))


class StepWatchdog:
    def __init__(self, rank: int, timeout_s: float | None = None, describe=None, poll_s: float | None = None,
                 exit_fn=None):
        self.rank = rank
        self.timeout_s = default_timeout() if timeout_s is None else float(timeout_s)
        self.describe = describe or (lambda: {})
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(5.0, self.timeout_s / 10))
        self.exit_fn = exit_fn or (lambda code: os._exit(code))
        self._open: deque = deque()  # [step, t_begin, event or None, host_done]
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.fired: str | None = None
        self._thread = None
        if self.timeout_s > 0:
            self._thread = threading.Thread(target=self._run, name=f"dllm-step-watchdog-r{rank}", daemon=True)
            self._thread.start()

    @property
    def enabled(self) -> bool:
        return self._thread is not None

    def begin(self, step: int):
        if not self.enabled:
            return
        with self._lock:
            self._open.append([step, time.monotonic(), None, False])

    def end(self, device: torch.device | None = None):
        """The step's host work is issued; on the GPU its completion is the event recorded here."""
        if not self.enabled:
            return
        ev = None
        if device is not None and device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        with self._lock:
            for rec in reversed(self._open):
                if rec[2] is None and not rec[3]:
                    rec[2], rec[3] = ev, ev is None
                    break

    def _done(self, rec) -> bool:
        if rec[3]:
            return True
        ev = rec[2]
        return ev is not None and ev.query()

    def _run(self):
        while not self._stop.wait(self.poll_s):
            with self._lock:
                while self._open and self._done(self._open[0]):
                    self._open.popleft()
                head = self._open[0] if self._open else None
            if head is None or time.monotonic() - head[1] < self.timeout_s:
                continue
            try:
                where = self.describe()
            except Exception as e:  # noqa: BLE001 - the report must not die on a broken describe()
                where = {"describe_error": repr(e)}
            state = "host still inside the step" if head[2] is None and not head[3] else "device has not finished it"
            self.fired = (f"[dllm watchdog] rank {self.rank}: step {head[0]} not finished after {self.timeout_s:.0f} s "
                          f"({state}); {where}")
            print(self.fired, file=sys.stderr, flush=True)
            self.exit_fn(EXIT_STALL)
            return

    def close(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2 * self.poll_s + 1)
            self._thread = None
