"""Loop overhead of the entry points: the same tokenised synthetic SAMSum batches through (a) the engine alone on
batches pre-staged on the GPU and (b) the full data path (DataLoader + collate + pinned H2D + engine step), at the
same per-GPU batch.  The entry points' own steady-state numbers (train_steady_samples_per_second) include the rest of
their loops; (b) / (a) isolates what the data path costs.

    python tools/loop_overhead.py --model t5-base --batch 128 --steps 10
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llms_example_amd.cli import base_parser, build_data, model_config  # noqa: E402
from distributed_llms_example_amd.data.collator import DataCollatorForSeq2Seq  # noqa: E402
from distributed_llms_example_amd.models import build_model  # noqa: E402
from distributed_llms_example_amd.parallel.env import init_distributed  # noqa: E402
from distributed_llms_example_amd.train.engine import TrainEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="t5-base")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    args = base_parser("x").parse_args(["--model-ckpt", a.model, "--synthetic", str(a.batch * (a.steps + 3))])
    cfg = model_config(args)
    tok, tr, _ = build_data(args, cfg)
    env = init_distributed()
    torch.manual_seed(0)
    eng = TrainEngine(build_model(cfg), env, lr=5e-5, weight_decay=0.01, dtype=torch.bfloat16).train()
    coll = DataCollatorForSeq2Seq.for_model(cfg)
    dl = torch.utils.data.DataLoader(tr, batch_size=a.batch, shuffle=False, collate_fn=coll, pin_memory=True)
    staged = [{k: v.to(env.device) for k, v in b.items()} for _, b in zip(range(a.steps + 3), dl)]
    res = {}
    for mode in ("engine_prestaged", "dataloader_h2d"):
        it = iter(dl)
        for i in range(3 + a.steps):
            if i == 3:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            if mode == "engine_prestaged":
                b = staged[i]
            else:
                b = {k: v.to(env.device, non_blocking=True) for k, v in next(it).items()}
            eng.forward_backward(b)
            eng.step()
        torch.cuda.synchronize()
        res[mode] = a.batch * a.steps / (time.perf_counter() - t0)
    res["overhead_pct"] = round(100 * (res["engine_prestaged"] / res["dataloader_h2d"] - 1), 2)
    mean_len = float(tr.attention_mask[: a.batch * a.steps].sum(1).mean())
    print(json.dumps({"model": a.model, "batch": a.batch, "steps": a.steps, "mean_src_tokens": round(mean_len, 1),
                      **{k: round(v, 2) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
