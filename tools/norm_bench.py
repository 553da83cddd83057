"""Fused residual + dropout + RMSNorm kernels (csrc/norm.hip) at the t5-base b=512 shapes: time and HBM rate.

    python tools/norm_bench.py            # the t5-base b=512 shapes
    python tools/norm_bench.py --rows 4096,1024 --partials   # micro-batch shapes of a deferred GA window

Bytes counted: forward reads x + resid, writes out + s; backward reads dout + ds_extra + s, writes dx + dstream.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(rows_list, d, reps, partials=False):
    import torch
    from distributed_llms_example_amd import _ext
    C = _ext.native()
    out = []
    for N in rows_list:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(N, d, device="cuda", generator=g).bfloat16()
        r = torch.randn(N, d, device="cuda", generator=g).bfloat16()
        w = torch.rand(d, device="cuda", generator=g).bfloat16() + 0.5
        dout = torch.randn(N, d, device="cuda", generator=g).bfloat16()
        dse = torch.randn(N, d, device="cuda", generator=g).bfloat16()
        fwd = lambda: C.norm_fwd(x, r, w, None, 1e-6, 0.1, 7, 0, True)
        o, s, mean, rstd = fwd()
        bwd = lambda: C.norm_bwd(dout, dse, s, w, None, mean, rstd, 0.1, 7, 0, True, None, None,
                                 partials_only=partials)
        res = {"N": N, "d": d, "G": 512, "partials_only": partials}
        for name, fn, nbytes in (("fwd", fwd, 4 * N * d * 2), ("bwd", bwd, 5 * N * d * 2)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            res[name + "_us"] = round(ms * 1e3, 1)
            res[name + "_TBps"] = round(nbytes / (ms * 1e-3) / 1e12, 2)
        out.append(res)
        print(json.dumps(res), flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="524288,65536")
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--partials", action="store_true", help="backward keeps the per-block dw partials (deferred GA)")
    a = ap.parse_args()
    rows = [int(v) for v in a.rows.split(",")]
    one(rows, a.d, a.reps, a.partials)


if __name__ == "__main__":
    main()
