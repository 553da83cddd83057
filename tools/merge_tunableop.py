#!/usr/bin/env python
"""Merge TunableOp result files (written by ``DLLM_TUNABLEOP=tune``) into the in-tree table.

    python tools/merge_tunableop.py gpurun_out/tune/*.csv [-o configs/tunableop/gfx950.csv]

Validator lines come from the first input that has them (they must match the running stack); solution
lines are keyed by (op, shape) and later files win, so a re-tune overrides an older pick.
"""
from __future__ import annotations

import argparse
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read(path):
    val, sol = {}, {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            parts = line.split(",")
            if parts[0] == "Validator":
                val[parts[1]] = line
            elif len(parts) >= 3:
                sol[(parts[0], parts[1])] = line
    return val, sol


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("-o", "--out", default=os.path.join(ROOT, "configs", "tunableop", "gfx950.csv"))
    a = ap.parse_args()
    val, sol = read(a.out) if os.path.exists(a.out) else ({}, {})
    n0 = len(sol)
    for p in a.inputs:
        v, s = read(p)
        for k, line in v.items():
            val.setdefault(k, line)
        sol.update(s)
    with open(a.out, "w") as f:
        for line in val.values():
            f.write(line + "\n")
        for k in sorted(sol):
            f.write(sol[k] + "\n")
    print(f"{a.out}: {n0} -> {len(sol)} solutions")


if __name__ == "__main__":
    main()
