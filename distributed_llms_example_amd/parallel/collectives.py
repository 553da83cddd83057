"""Collectives used outside the gradient path (metrics, generation results, barriers).

Equivalents of the Accelerate / raw-dist helpers the reference calls:
``gather`` (C7/C9: all_gather_into_tensor, accelerate/utils/operations.py:322-358),
``pad_across_processes`` (C8, operations.py:780-781), ``mean_across_processes`` (R7/R11 metric sync),
``barrier`` (C10).  On one process they are identities.  Tensors stay on their device (RCCL on GPU).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _ws(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def gather(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate ``t`` from every rank along dim 0 (all ranks must pass the same shape)."""
    ws = _ws(group)
    if ws == 1:
        return t
    if t.dim() == 0:
        t = t.reshape(1)
    out = torch.empty((ws * t.shape[0], *t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def gather_dict(d: dict, group=None) -> dict:
    return {k: gather(v, group) for k, v in d.items()}


def pad_across_processes(t: torch.Tensor, dim: int = 1, pad_index: int = 0, pad_first: bool = False,
                         group=None) -> torch.Tensor:
    """Pad ``dim`` to the max size over ranks (one all_gather of the shape, as Accelerate does)."""
    ws = _ws(group)
    if ws == 1:
        return t
    size = torch.tensor([t.shape[dim]], device=t.device, dtype=torch.int64)
    sizes = gather(size, group)
    m = int(sizes.max().item())
    if m == t.shape[dim]:
        return t
    shape = list(t.shape)
    shape[dim] = m
    out = t.new_full(shape, pad_index)
    idx = [slice(None)] * t.dim()
    idx[dim] = slice(m - t.shape[dim], m) if pad_first else slice(0, t.shape[dim])
    out[tuple(idx)] = t
    return out


def mean_across_processes(values: dict, device, group=None, skip=("epoch",)) -> dict:
    """Gather scalar metrics from every rank and average them (keys in ``skip`` keep rank 0's value)."""
    keys = sorted(values)
    t = torch.tensor([float(values[k]) for k in keys], device=device, dtype=torch.float64)
    ws = _ws(group)
    if ws > 1:
        g = torch.empty(ws * len(keys), device=device, dtype=torch.float64)
        dist.all_gather_into_tensor(g, t, group=group)
        g = g.view(ws, len(keys))
    else:
        g = t.view(1, -1)
    out = {}
    for i, k in enumerate(keys):
        out[k] = int(g[0, i].item()) if k in skip else float(g[:, i].mean().item())
    return out


def all_reduce_sum(t: torch.Tensor, group=None) -> torch.Tensor:
    if _ws(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


def broadcast_object(obj, src: int = 0, group=None):
    if _ws(group) == 1:
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=group)
    return lst[0]


def barrier(group=None, device=None):
    if _ws(group) > 1:
        if device is not None and device.type == "cuda":
            dist.barrier(group=group, device_ids=[device.index])
        else:
            dist.barrier(group=group)
