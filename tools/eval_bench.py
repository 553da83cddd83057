"""Eval-generation throughput: ``generate(num_beams=2, max_length=128)`` over 818 SAMSum-test-shaped samples
(ref/train-accelerator.py:239-249).  Modes: ``fused`` = device-side beam bookkeeping with the one-kernel beam step
(csrc/beam.hip), ``device`` = the same with the torch composite step (DLLM_ROUTE gen_fused_beam=0), ``host`` = the
per-step host loop (gen_host=1).

    python tools/eval_bench.py [--model t5-base] [--batch 64] [--src-len 512] [--n 818] [--modes fused,device,host]
Synthetic prompts (random ids, ragged attention masks) and random-init weights; prints one JSON line per mode.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llms_example_amd.models import build_model, resolve_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="t5-base")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--src-len", type=int, default=512)
    ap.add_argument("--n", type=int, default=818)
    ap.add_argument("--beams", type=int, default=2)
    ap.add_argument("--max-length", type=int, default=128)
    ap.add_argument("--modes", default="fused,device,host")
    a = ap.parse_args()
    torch.manual_seed(0)
    cfg = resolve_config(a.model)
    m = build_model(cfg).cuda().to(torch.bfloat16).eval()
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(3, cfg.vocab_size, (a.n, a.src_len), generator=g)
    lens = torch.randint(a.src_len // 4, a.src_len + 1, (a.n,), generator=g)
    am = (torch.arange(a.src_len)[None, :] < lens[:, None]).long()
    for mode in a.modes.split(","):
        os.environ["DLLM_ROUTE"] = (f"gen_host={1 if mode == 'host' else 0},"
                                    f"gen_fused_beam={1 if mode == 'fused' else 0}")
        m.generate(ids[:a.batch].cuda(), attention_mask=am[:a.batch].cuda(), max_length=8, num_beams=a.beams)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        toks = 0
        for i in range(0, a.n, a.batch):
            out = m.generate(ids[i:i + a.batch].cuda(), attention_mask=am[i:i + a.batch].cuda(),
                             max_length=a.max_length, num_beams=a.beams)
            toks += out.numel()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"mode": mode, "model": a.model, "samples": a.n, "batch": a.batch, "num_beams": a.beams,
                          "max_length": a.max_length, "src_len": a.src_len, "seconds": round(dt, 3),
                          "samples_per_s": round(a.n / dt, 2), "gen_tokens": toks}), flush=True)


if __name__ == "__main__":
    main()
