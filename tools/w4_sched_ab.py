"""A/B of two csrc/gemm_w4.hip k-loop schedules (DLLM_ROUTE w4_sched, read per launch) on every mode the t5-base b=512 step
runs: NT forward, NN input gradient, weight gradient (split-K), ReLU FFN forward (bit mask) and its backward.
Interleaved rounds in one process, median, random operands (cdna_hip_programming.md §5.4 rules 24-25).

    python tools/w4_sched_ab.py [--rs-a 1] [--rs-b 257] [--rounds 5] [--iters 10] [--batch 128]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llms_example_amd import _ext  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rs-a", default="1")
    ap.add_argument("--rs-b", default="257")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    C = _ext.native()
    assert C is not None, f"native extension not loaded: {_ext.load_error()}"
    T = 1024 * a.batch
    r = lambda *s: torch.randn(*s, device="cuda").to(torch.bfloat16)  # noqa: E731
    x768, w2304, w768, wi, wo = r(T, 768), r(2304, 768) * 0.03, r(768, 768) * 0.03, r(3072, 768) * 0.03, r(768, 3072) * 0.02
    dy2304, dy768, h3072 = r(T, 2304), r(T, 768), r(T, 3072)
    mask = torch.empty(C.gemm_w4_mask_words(T, 3072), device="cuda", dtype=torch.int32)
    g2304 = torch.zeros(2304, 768, device="cuda", dtype=torch.float32)
    g768 = torch.zeros(768, 3072, device="cuda", dtype=torch.float32)
    cases = {
        "fwd qkv   (K 768, N 2304)": (2 * T * 768 * 2304, lambda: C.gemm_w4(x768, w2304, False)),
        "fwd o     (K 768, N 768)": (2 * T * 768 * 768, lambda: C.gemm_w4(x768, w768, False)),
        "dgrad qkv (K 2304, N 768)": (2 * T * 768 * 2304, lambda: C.gemm_w4(dy2304, w2304, True)),
        "dgrad wo  (K 768, N 3072)": (2 * T * 768 * 3072, lambda: C.gemm_w4(dy768, wo, True)),
        "wgrad qkv (2304 x 768)": (2 * T * 768 * 2304, lambda: C.gemm_wgrad(dy2304, x768, g2304, True, -1, 0)),
        "wgrad wo  (768 x 3072)": (2 * T * 768 * 3072, lambda: C.gemm_wgrad(dy768, h3072, g768, True, -1, 0)),
        "relu ffn fwd (wi)": (2 * T * 768 * 3072,
                              lambda: C.gemm_w4(x768, wi, False, None, None, False, -1, True, 1, 0.1, 7, mask)),
        "drelu ffn bwd (wo)": (2 * T * 768 * 3072,
                               lambda: C.gemm_w4(dy768, wo, True, None, None, False, -1, True, 7, 0.1, 7, mask)),
    }
    # outputs of the two schedules must be bit-identical (same products, same order)
    for name, (_, fn) in cases.items():
        if name.startswith("wgrad"):
            continue
        os.environ["DLLM_ROUTE"] = "w4_sched=" + a.rs_a
        ra = fn().clone()
        os.environ["DLLM_ROUTE"] = "w4_sched=" + a.rs_b
        rb = fn().clone()
        assert torch.equal(ra, rb), f"{name}: schedules disagree"
    print(f"# w4 schedules RS={a.rs_a} (A) vs RS={a.rs_b} (B), tokens {T}, median of {a.rounds} interleaved rounds; "
          f"outputs bit-identical", flush=True)
    tot = {"A": 0.0, "B": 0.0}
    for name, (fl, fn) in cases.items():
        ts = {"A": [], "B": []}
        for _ in range(a.rounds):
            for arm, rs in (("A", a.rs_a), ("B", a.rs_b)):
                os.environ["DLLM_ROUTE"] = "w4_sched=" + rs
                ts[arm].append(timeit(fn, a.iters))
        ma, mb = statistics.median(ts["A"]), statistics.median(ts["B"])
        tot["A"] += ma
        tot["B"] += mb
        print(f"{name:28s} A {ma * 1e6:9.1f} us {fl / ma / 1e12:7.1f} TF/s   B {mb * 1e6:9.1f} us {fl / mb / 1e12:7.1f} TF/s"
              f"   B/A {mb / ma:.4f}", flush=True)
    print(f"{'sum':28s} A {tot['A'] * 1e6:9.1f} us   B {tot['B'] * 1e6:9.1f} us   B/A {tot['B'] / tot['A']:.4f}")


if __name__ == "__main__":
    main()
