"""Per-dispatch-shape breakdown of a rocprofv3 --kernel-trace run: time per (kernel, grid) group, so that e.g. every
hipBLASLt / hand-written GEMM shape of a training step shows its own in-situ time (the --stats view only has per-name
averages).  Reads the rocpd SQLite database (rocprofv3 >= 7) or a kernel_trace.csv.

    python tools/trace_shapes.py <run.db | kernel_trace.csv> <steps> [top]
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def _rows(path):
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        cur = con.execute("select * from kernels limit 1")
        cols = [d[0] for d in cur.description]
        want = [c for c in cols if c.lower() in ("name", "duration", "grid_size_x", "grid_size_y", "grid_size_z",
                                                   "grid_x", "grid_y", "grid_z", "workgroup_size_x", "grid_size")]
        for r in con.execute(f"select {', '.join(want)} from kernels"):
            d = dict(zip(want, r))
            g = tuple(d.get(k) for k in want if k.lower().startswith("grid"))
            wg = d.get("workgroup_size_x")
            yield d["name"], float(d["duration"]), g, wg
    else:
        for r in csv.DictReader(open(path)):
            g = (r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z"))
            yield r["Kernel_Name"], float(r["End_Timestamp"]) - float(r["Start_Timestamp"]), g, r.get("Workgroup_Size_X")


def main(path, steps, top=40):
    agg = defaultdict(lambda: [0, 0.0])
    tot = 0.0
    for name, dur, g, wg in _rows(path):
        a = agg[(name[:90], g, wg)]
        a[0] += 1
        a[1] += dur
        tot += dur
    print(f"total {tot / steps / 1e6:.2f} ms/step over {steps} steps; {len(agg)} (kernel, grid) groups")
    for (name, g, wg), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / steps / 1e6:8.2f} ms/step {100 * t / tot:5.1f}%  calls/step {n / steps:5.1f}  avg {t / n / 1e3:8.1f} us"
              f"  grid {g} wg {wg}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 40)
