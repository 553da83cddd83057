"""Per-kernel averages of rocprofv3 --pmc counters from the rocpd SQLite output (one row per kernel family)."""
import sqlite3
import sys
from collections import defaultdict


def main(paths):
    agg = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for p in paths:
        c = sqlite3.connect(p)
        for name, cnt, val, d, disp in c.execute(
                "select kernel_name, counter_name, value, duration, dispatch_id from counters_collection"):
            key = name[:70]
            agg[key][cnt].append(val)
            dur[key].append((disp, d))
    for k, cs in agg.items():
        if "rocclr" in k or "elementwise" in k or "distribution" in k:
            continue
        ds = sorted(set(dur[k]))
        us = sum(d for _, d in ds) / len(ds) / 1e3
        print(f"== {k}  ({len(ds)} dispatches, {us:.1f} us avg)")
        for cn, vs in sorted(cs.items()):
            print(f"   {cn:28s} {sum(vs) / len(vs):16.1f}")


if __name__ == "__main__":
    main(sys.argv[1:])
