"""Valohai platform integration (``valohai-utils`` is not installed here; this is a compatible shim).

* ``inputs(name).path()`` → first file under ``<root>/inputs/<name>/`` (ref/train-torchrun.py:151-152)
* ``outputs().path(p)`` → ``<root>/outputs/<p>`` (created) (ref/helpers.py:26)
* ``distributed.master().primary_local_ip``, ``distributed.required_count``, ``distributed.me().rank``
  (ref/train-task.py:421-425) — read from ``/valohai/config/distributed.json`` when present, else env
  ``VH_MASTER_IP`` / ``VH_WORLD_SIZE`` / ``VH_RANK`` (tests, or one node of 8×MI355X where the
  "machines" are local processes).
* ``save_valohai_metadata(model, output_dir)`` / ``get_run_identification()`` (ref/helpers.py:12-40):
  HF-format save + one ``<file>.metadata.json`` sidecar per output file with the dataset-version URI,
  alias and tags.  Differences from the reference: only rank 0 writes, and
  sidecars are not written for sidecars.

The root is ``/valohai`` unless ``VH_ROOT`` overrides it.
"""
from __future__ import annotations

import datetime
import json
import os
import time


def root() -> str:
    return os.environ.get("VH_ROOT", "/valohai")


class _Input:
    def __init__(self, name):
        self.name = name

    def dir_path(self) -> str:
        return os.path.join(root(), "inputs", self.name)

    def paths(self):
        d = self.dir_path()
        if not os.path.isdir(d):
            return []
        return [os.path.join(d, f) for f in sorted(os.listdir(d))]

    def path(self, default=None) -> str:
        ps = self.paths()
        if ps:
            return ps[0]
        if default is not None:
            return default
        return os.path.join(self.dir_path(), "MISSING")


def inputs(name: str) -> _Input:
    return _Input(name)


class _Outputs:
    def __init__(self, sub: str | None = None):
        self.sub = sub

    def dir_path(self) -> str:
        return os.path.join(root(), "outputs")

    def path(self, p: str) -> str:
        full = p if os.path.isabs(p) else os.path.join(self.dir_path(), p)
        parent = full if not os.path.splitext(full)[1] else os.path.dirname(full)
        os.makedirs(parent, exist_ok=True)
        return full


def outputs(sub: str | None = None) -> _Outputs:
    return _Outputs(sub)


class _Member:
    def __init__(self, rank, ip):
        self.rank = rank
        self.primary_local_ip = ip


class _Distributed:
    def _cfg(self):
        p = os.path.join(root(), "config", "distributed.json")
        if os.path.exists(p):
            with open(p) as f:
                return json.load(f)
        return None

    @property
    def required_count(self) -> int:
        c = self._cfg()
        if c and "required_count" in c:
            return int(c["required_count"])
        return int(os.environ.get("VH_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))

    def me(self) -> _Member:
        c = self._cfg()
        if c and "me" in c:
            return _Member(int(c["me"]["rank"]), c["me"].get("primary_local_ip", "127.0.0.1"))
        return _Member(int(os.environ.get("VH_RANK", os.environ.get("RANK", "0"))), "127.0.0.1")

    def master(self) -> _Member:
        c = self._cfg()
        if c and "master" in c:
            return _Member(0, c["master"]["primary_local_ip"])
        return _Member(0, os.environ.get("VH_MASTER_IP", os.environ.get("MASTER_ADDR", "127.0.0.1")))

    @property
    def is_distributed_task(self) -> bool:
        return self.required_count > 1


distributed = _Distributed()


def get_run_identification():
    """(project_name, execution_id) from /valohai/config/execution.json, else ('test', <unix time>)."""
    try:
        with open(os.path.join(root(), "config", "execution.json")) as f:
            d = json.load(f)
        return d["valohai.project-name"].split("/")[1], d["valohai.execution-id"]
    except (FileNotFoundError, KeyError, IndexError):
        return "test", str(int(time.time()))


def write_metadata_sidecars(output_dir: str, project_name: str | None = None, exec_id: str | None = None):
    if project_name is None or exec_id is None:
        project_name, exec_id = get_run_identification()
    meta = {"valohai.dataset-versions": [{
        "uri": f"dataset://llm-models/{project_name}_{exec_id}",
        "targeting_aliases": [f"dev-{datetime.date.today()}-model"],
        "valohai.tags": ["dev", "llm"],
    }]}
    written = []
    for f in sorted(os.listdir(output_dir)):
        if f.endswith(".metadata.json") or os.path.isdir(os.path.join(output_dir, f)):
            continue
        p = os.path.join(output_dir, f"{f}.metadata.json")
        with open(p, "w") as fh:
            json.dump(meta, fh)
        written.append(p)
    return written


def save_valohai_metadata(model, output_dir: str, is_main_process: bool = True, tokenizer=None):
    """ref/helpers.py:12-28: save the model (HF format) and write per-file metadata sidecars."""
    if not is_main_process:
        return []
    from ..models.hf_io import save_pretrained
    save_pretrained(model, output_dir)
    if tokenizer is not None and hasattr(tokenizer, "save_pretrained"):
        tokenizer.save_pretrained(output_dir)
    return write_metadata_sidecars(output_dir)
