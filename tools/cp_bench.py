#!/usr/bin/env python
"""Context-parallel attention compute on one MI355X: per-rank cost of the ring blocks vs the unsharded op.

For a global encoder length N split over W ranks, one CP rank runs W blocks of (N/W x N/W) flash attention
forward + backward (parallel/context.py) plus the LSE merges.  This times rank 0's share (W blocks of
its query shard against every K/V shard, no communication: on a node the K/V transfer of the next block
overlaps the current block) and compares W x that with the monolithic (N x N) kernel, i.e. the compute
efficiency of sharding.  T5 shapes: H heads of 64, relative bias, dropout 0.1 off/on.

    python tools/cp_bench.py [--n 8192,16384] [--w 1,2,4,8] [--heads 32] [--batch 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_llms_example_amd import _ext  # noqa: E402
from distributed_llms_example_amd.ops import attention as A  # noqa: E402
from distributed_llms_example_amd.parallel import context as cp  # noqa: E402


def _time(fn, iters=5, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        fn()
    t1.record()
    torch.cuda.synchronize()
    return t0.elapsed_time(t1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="8192,16384")
    ap.add_argument("--w", default="1,2,4,8")
    ap.add_argument("--heads", type=int, default=32)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--p", type=float, default=0.0)
    a = ap.parse_args()
    assert torch.cuda.is_available() and _ext.native() is not None
    dev = "cuda"
    B, H, D = a.batch, a.heads, 64
    for N in (int(x) for x in a.n.split(",")):
        q, k, v, do = (torch.randn(B, N, H, D, device=dev).to(torch.bfloat16) for _ in range(4))
        table = torch.randn(32, H, device=dev) * 0.5
        lut = A.relative_bias_lut(table, N, N, True, 32, 128)

        def mono():
            qq, kk, vv = (t.detach().requires_grad_(True) for t in (q, k, v))
            o = A.attention(qq, kk, vv, bias_lut=lut, dropout_p=a.p, seed=1)
            o.backward(do)
        try:
            t_mono = _time(mono)
        except RuntimeError as e:  # the single-kernel path stages per-key state in LDS: bounded length
            print(json.dumps({"N": N, "mono": f"unsupported ({e})"}), flush=True)
            t_mono = None
        for W in (int(x) for x in a.w.split(",")):
            if N % W:
                continue
            S = N // W
            luts = [A.relative_bias_lut(table, S, S, True, 32, 128, q_offset=(0 - s) * S) for s in range(W)]
            qr, dor = q[:, :S], do[:, :S].contiguous()

            def rank0():
                o_acc = l_acc = None
                masks = []
                for s in range(W):
                    o_b, l_b, dm = cp._block_fwd(qr, k[:, s * S:(s + 1) * S], v[:, s * S:(s + 1) * S], None, luts[s],
                                                 luts[s]._dllm_sat, 1.0, a.p, cp._block_seed(1, 0, s))
                    masks.append(dm)
                    o_acc, l_acc = (o_b, l_b) if o_acc is None else cp._merge(o_acc, l_acc, o_b, l_b)
                o = o_acc.to(torch.bfloat16)
                lse = l_acc.contiguous()
                dq = torch.zeros(B, S, H, D, device=dev)
                for s in range(W):
                    r = cp._block_bwd(dor, qr, k[:, s * S:(s + 1) * S], v[:, s * S:(s + 1) * S], o, lse, None,
                                      luts[s], luts[s]._dllm_sat, 1.0, a.p, cp._block_seed(1, 0, s), True, masks[s])
                    dq += r[0]
            try:
                t_rank = _time(rank0)
            except RuntimeError as e:
                print(json.dumps({"N": N, "W": W, "rank": f"unsupported ({e})"}), flush=True)
                continue
            flops = 4 * B * H * N * N * D * 3.5 / W  # fwd 2 GEMMs + bwd 5 GEMMs (x0.5 fwd-equivalent units)
            print(json.dumps({"N": N, "W": W, "heads": H, "batch": B, "p": a.p,
                              "mono_ms": round(t_mono, 3) if t_mono else None, "rank_ms": round(t_rank, 3),
                              "ideal_rank_ms": round(t_mono / W, 3) if t_mono else None,
                              "efficiency": round(t_mono / W / t_rank, 3) if t_mono else None,
                              "rank_tflops": round(flops / t_rank / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
