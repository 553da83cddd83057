"""Process bootstrap: one process per GPU, torch.distributed over RCCL (backend "nccl" on ROCm).

Three launch contracts the reference uses:

* torchrun / ``accelerate launch`` → env ``RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT``
  (torch/distributed/elastic/agent/server/local_elastic_agent.py:305-322);
* train-task → ``init_method=tcp://<master_ip>:1234`` with rank/world from the Valohai distributed
  API (ref/train-task.py:404-430), here also from ``platform/valohai.py``;
* nothing set → single process, world 1 (Accelerate's ``DistributedType.NO``, state.py:177-316).

Backend: ``nccl`` (= RCCL over xGMI) when GPUs are present, ``gloo`` on CPU (tests).  The device is
``cuda:LOCAL_RANK``; ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is kept for RCCL's dmabuf IPC.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main_process(self) -> bool:
        return self.rank == 0

    @property
    def is_local_main_process(self) -> bool:
        return self.local_rank == 0

    def barrier(self):
        if self.is_distributed and dist.is_initialized():
            if self.backend == "nccl":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()


_ENV: DistEnv | None = None


def _pick_backend(use_gpu: bool) -> str:
    # DLLM_DIST_BACKEND=gloo lets several ranks share one GPU (RCCL refuses duplicate devices): used to
    # rehearse the multi-process GPU path on a 1-GPU box.
    return os.environ.get("DLLM_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")


def init_distributed(init_method: str | None = None, rank: int | None = None, world_size: int | None = None,
                     backend: str | None = None, timeout_s: float = 1800.0, cpu: bool | None = None) -> DistEnv:
    """Initialise (once) and return the process's :class:`DistEnv`.  ``timeout_s`` = HF
    ``ddp_timeout`` default (training_args.py:658)."""
    global _ENV
    if _ENV is not None:
        return _ENV
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    use_gpu = torch.cuda.is_available() if cpu is None else not cpu
    if os.environ.get("DLLM_FORCE_CPU", "0") == "1":
        use_gpu = False
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    ws = world_size if world_size is not None else env_world
    rk = rank if rank is not None else int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rk if init_method else 0)))
    local_ws = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws if init_method is None else 1)))
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev_index = local_rank % max(ndev, 1)
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
        from ..utils import tunableop
        tunableop.enable(dev_index)
    else:
        device = torch.device("cpu")
    be = backend or _pick_backend(use_gpu)
    if ws > 1 and not dist.is_initialized():
        kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if init_method is not None:
            kw.update(init_method=init_method, rank=rk, world_size=ws)
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    if dist.is_initialized():  # a process group set up by the caller (or just now) is the truth
        rk = dist.get_rank()
        ws = dist.get_world_size()
        be = dist.get_backend()
    _ENV = DistEnv(rank=rk, world_size=ws, local_rank=local_rank, local_world_size=local_ws,
                   backend=be if ws > 1 else "none", device=device)
    return _ENV


def get_env() -> DistEnv:
    return _ENV if _ENV is not None else init_distributed()


def shutdown():
    global _ENV
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass
    _ENV = None
