"""Summarise a rocprofv3 --stats kernel CSV: per-step time by kernel (and grouped families)."""
import csv
import re
import sys
from collections import defaultdict


def family(name):
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        return "GEMM (hipBLASLt)"
    m = re.search(r"\b(attn_\w+|norm_\w+|act_\w+|ce_\w+|adamw\w*|col_sum\w*|colsum\w*|sq_norm\w*|dropout\w*|"
                  r"sum_partials|gemm_wgrad\w*|splitk_reduce\w*)", name)
    if m:
        return m.group(1)
    m = re.search(r"at::native::(\w+)", name)
    return "torch:" + (m.group(1) if m else name[:40])


def _rows_from_db(path):
    """rocprofv3 >= 7 writes a rocpd SQLite database; aggregate its ``kernels`` view like --stats does."""
    import sqlite3
    agg = defaultdict(lambda: [0, 0.0])
    for name, dur in sqlite3.connect(path).execute("select name, duration from kernels"):
        a = agg[name]
        a[0] += 1
        a[1] += float(dur)
    return [{"Name": k, "Calls": n, "TotalDurationNs": t, "AverageNs": t / n} for k, (n, t) in agg.items()]


def main(path, steps):
    rows = _rows_from_db(path) if path.endswith(".db") else list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    fam = defaultdict(float)
    for r in rows:
        fam[family(r["Name"])] += float(r["TotalDurationNs"])
    print(f"total GPU kernel time {tot/1e6:.1f} ms over {steps} steps = {tot/steps/1e6:.2f} ms/step")
    print("--- by family (ms/step, %)")
    for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
        print(f"{v/steps/1e6:9.2f}  {100*v/tot:5.1f}%  {k}")
    print("--- top kernels")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        print(f"{float(r['TotalDurationNs'])/steps/1e6:9.2f} ms/step  calls/step {int(r['Calls'])/steps:6.1f}  "
              f"avg {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:100]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
