"""AdamW kernel variants over a BART-large-sized flat buffer (406 M params, bf16 params, fp32 master / grads / moments):
v1 (4 elements / thread) vs the 8-wide kernel with and without nontemporal access, several grid sizes."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llms_example_amd import _ext  # noqa: E402

n = 406_000_000 // 64 * 64
dev = "cuda"
p = torch.randn(n, device=dev).to(torch.bfloat16)
master = p.float()
g = torch.randn(n, device=dev) * 1e-3
m = torch.zeros(n, device=dev)
v = torch.zeros(n, device=dev)
mask = torch.ones(n, dtype=torch.uint8, device=dev)
coef = torch.ones((), device=dev)
C = _ext.native()
variants = [("v1", {"DLLM_ADAMW_V1": "1"})] + [
    (f"v8 nt={nt} grid={gr}", {"DLLM_ADAMW_NT": nt, "DLLM_ADAMW_GRID": gr}) for nt in ("0", "1")
    for gr in ("1024", "2048", "4096", "8192")]
for rep in range(2):
    for name, env in variants:
        for k in ("DLLM_ADAMW_V1", "DLLM_ADAMW_NT", "DLLM_ADAMW_GRID"):
            os.environ.pop(k, None)
        os.environ.update(env)
        for _ in range(2):
            C.adamw_step(p, master, g, m, v, mask, coef, 1e-4, 0.9, 0.999, 1e-8, 0.01, 0.1, 0.001)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            C.adamw_step(p, master, g, m, v, mask, coef, 1e-4, 0.9, 0.999, 1e-8, 0.01, 0.1, 0.001)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        print(json.dumps({"variant": name, "ms": round(dt * 1e3, 3), "GB_per_s": round(n * 21 / dt / 1e9, 1)}),
              flush=True)
