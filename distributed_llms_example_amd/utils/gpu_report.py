"""Environment report (replaces ``print_gpu_report``, ref/train-torchrun.py:37-58, which spawns
``nvidia-smi`` and calls ``torch.cuda.current_device()`` unconditionally — both fail on ROCm / CPU,
SURVEY.md Appendix A Q1).  ROCm-aware and safe on CPU; uses ``amd-smi`` / ``rocm-smi`` only if present.
"""
from __future__ import annotations

import shutil
import subprocess
import sys

import torch


def gpu_report(device=None, print_fn=print, run_smi: bool = False) -> dict:
    info = {"python": sys.version.split()[0], "torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
            "device_count": torch.cuda.device_count() if torch.cuda.is_available() else 0, "device": str(device)}
    if torch.cuda.is_available():
        idx = device.index if (device is not None and getattr(device, "index", None) is not None) \
            else torch.cuda.current_device()
        p = torch.cuda.get_device_properties(idx)
        info.update({"name": p.name, "arch": getattr(p, "gcnArchName", ""), "total_memory_gb": round(
            p.total_memory / 2**30, 1), "compute_units": p.multi_processor_count, "current_device": idx})
    for k, v in info.items():
        print_fn(f"__{k}: {v}")
    if run_smi:
        for tool, args in (("amd-smi", ["static", "--asic"]), ("rocm-smi", ["--showproductname"])):
            if shutil.which(tool):
                try:
                    out = subprocess.run([tool] + args, capture_output=True, text=True, timeout=20)
                    print_fn(out.stdout.strip()[:2000])
                except Exception as e:  # pragma: no cover
                    print_fn(f"{tool} failed: {e}")
                break
    return info
