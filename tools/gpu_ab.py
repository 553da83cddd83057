#!/usr/bin/env python
"""One parametrised GPU-box session: tests, interleaved A/B arms, bench lines and rocprofv3 summaries.

Replaces the per-experiment lease scripts of rounds 1-4.  Run on the GPU box (through gpurun), from the repo root:

    python tools/gpu_ab.py --tag r5a --tests "tests/test_kernels_gpu.py -k attn" \
        --bench "--steps 12 --warmup 3" --arms base=ab/base.so,new=distributed_llms_example_amd/_C*.so --reps 3 \
        --env-arms "lib=DLLM_ROUTE=proj_dgrad=lib,w4=DLLM_ROUTE=proj_dgrad=w4" --prof "--steps 2 --warmup 1 --graph off"

Steps, each under its own time limit; the session stops at the first failure (a GPU fault, a time limit, an abort):

* ``--tests``: ``pytest -m gpu`` over the given selection (one process);
* ``--bench`` x ``--reps``, interleaved over the arms: ``--arms name=path.so,...`` swaps the in-tree ``_C`` (the
  loader's ``DLLM_NATIVE_SO``), ``--env-arms name=K=V;K2=V2,...`` sets environment variables, ``--tree-arms
  name=dir,...`` runs another checkout's bench.py with its own package and library (e.g. the round-start tree built
  under ab/, tools/regression_gate.sh); one JSON bench line per run goes to ``<tag>/bench.jsonl`` with the arm name
  added, and a per-config table of median samples/s per arm (delta vs the first arm) closes the session;
* ``--prof``: ``rocprofv3 --kernel-trace --stats`` over ``bench.py <args>`` (first arm), summarised by
  tools/prof_summary.py (kernel families) and tools/trace_shapes.py (per-dispatch shapes) into ``<tag>/``;
* ``--cmd``: any extra command (e.g. a microbenchmark), output to ``<tag>/cmd.log``.

Everything lands in ``gpurun_out/<tag>/`` (merged back by gpurun); copy the summaries worth keeping to profiles/.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd: list[str], log: str, limit: int, env: dict | None = None, cwd: str = ROOT) -> int:
    """One GPU step under its own limit (timeout -k 10), output to ``log``; progress line on stdout."""
    t0 = time.time()
    with open(log, "w") as f:
        rc = subprocess.run(["timeout", "-k", "10", str(limit)] + cmd, stdout=f, stderr=subprocess.STDOUT,
                            env=env, cwd=cwd).returncode
    print(f"[gpu_ab] rc={rc} {time.time() - t0:7.1f}s  {' '.join(cmd)[:160]}", flush=True)
    return rc


def _arms(a) -> list[tuple[str, dict, str]]:
    """(name, environment additions, working tree) per arm."""
    arms = []
    for spec in filter(None, (a.tree_arms or "").split(",")):
        name, path = spec.split("=", 1)
        tree = path if os.path.isabs(path) else os.path.join(ROOT, path)
        if not os.path.exists(os.path.join(tree, "bench.py")):
            raise SystemExit(f"[gpu_ab] tree arm {name}: no bench.py under {tree}")
        arms.append((name, {}, tree))
    for spec in filter(None, (a.arms or "").split(",")):
        name, path = spec.split("=", 1)
        hits = glob.glob(os.path.join(ROOT, path)) if not os.path.isabs(path) else glob.glob(path)
        if not hits:
            raise SystemExit(f"[gpu_ab] arm {name}: no file matches {path}")
        arms.append((name, {"DLLM_NATIVE_SO": hits[0]}, ROOT))
    for spec in filter(None, (a.env_arms or "").split(",")):
        name, kvs = spec.split("=", 1)
        env = dict(kv.split("=", 1) for kv in filter(None, kvs.split(";")))
        arms.append((name, env, ROOT))
    return arms or [("default", {}, ROOT)]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--tests", default=None, help="pytest selection (run with -m gpu)")
    ap.add_argument("--tests-limit", type=int, default=900)
    ap.add_argument("--bench", action="append", default=[], help="bench.py arguments (repeatable: several configs)")
    ap.add_argument("--bench-limit", type=int, default=420)
    ap.add_argument("--arms", default=None, help="name=path.so,... (in-tree _C swapped per run)")
    ap.add_argument("--env-arms", default=None, help="name=K=V;K2=V2,... environment arms")
    ap.add_argument("--tree-arms", default=None, help="name=dir,... arms that run another checkout's bench.py")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--prof", action="append", default=[], help="bench.py arguments for a rocprofv3 kernel trace")
    ap.add_argument("--prof-limit", type=int, default=420)
    ap.add_argument("--cmd", action="append", default=[], help="extra command line (shell-split)")
    ap.add_argument("--cmd-limit", type=int, default=600)
    a = ap.parse_args()
    out = os.path.join(ROOT, "gpurun_out", a.tag)
    os.makedirs(out, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    base_env = dict(os.environ)
    arms = _arms(a)

    if a.tests:
        rc = _run([sys.executable, "-u", "-m", "pytest", "-q", "-m", "gpu", "--timeout", "240", "--timeout-method",
                   "thread", "-x"] + shlex.split(a.tests), os.path.join(out, "tests.log"), a.tests_limit)
        tail = open(os.path.join(out, "tests.log")).read().splitlines()[-15:]
        print("\n".join(tail), flush=True)
        if rc != 0:
            return rc

    for c, cmd in enumerate(a.cmd):
        rc = _run(shlex.split(cmd), os.path.join(out, f"cmd{c}.log"), a.cmd_limit)
        print("\n".join(open(os.path.join(out, f"cmd{c}.log")).read().splitlines()[-12:]), flush=True)
        if rc != 0:
            return rc

    lines = open(os.path.join(out, "bench.jsonl"), "a")
    results: dict = {}
    for rep in range(a.reps):
        for bi, bargs in enumerate(a.bench):
            for name, env, tree in arms:
                log = os.path.join(out, f"bench_{bi}_{name}_{rep}.log")
                rc = _run([sys.executable, "-u", "bench.py"] + shlex.split(bargs), log, a.bench_limit,
                          env=dict(base_env, **env), cwd=tree)
                if rc != 0:
                    print("\n".join(open(log).read().splitlines()[-20:]), flush=True)
                    return rc
                js = [ln for ln in open(log).read().splitlines() if ln.startswith("{") and '"metric"' in ln]
                if js:
                    d = json.loads(js[-1])
                    d.update({"arm": name, "rep": rep, "bench_args": bargs})
                    lines.write(json.dumps(d) + "\n")
                    lines.flush()
                    results.setdefault(bi, {}).setdefault(name, []).append(d["value"])
                    print(f"[gpu_ab] {name:>10s} rep {rep} cfg {bi}: {d['value']:9.2f} {d['unit']}  "
                          f"{d['ms_per_step']:9.3f} ms/step", flush=True)

    if results:
        _table(results, a.bench, [n for n, _, _ in arms], os.path.join(out, "bench_table.txt"))

    for pi, pargs in enumerate(a.prof):
        d = os.path.join(out, f"prof{pi}")
        os.makedirs(d, exist_ok=True)
        name, env, tree = arms[0]
        rc = _run(["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "run", "--", sys.executable, "bench.py"]
                  + shlex.split(pargs), os.path.join(out, f"prof{pi}.log"), a.prof_limit, env=dict(base_env, **env),
                  cwd=tree)
        if rc != 0:
            print("\n".join(open(os.path.join(out, f"prof{pi}.log")).read().splitlines()[-20:]), flush=True)
            return rc
        dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
        if dbs:
            steps = _prof_steps(pargs)
            for tool, fn in (("prof_summary.py", "summary"), ("trace_shapes.py", "shapes")):
                extra = ["60"] if tool == "trace_shapes.py" else []
                with open(os.path.join(out, f"{fn}{pi}.txt"), "w") as f:
                    subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool), dbs[0], str(steps)] + extra,
                                   stdout=f, stderr=subprocess.STDOUT, cwd=ROOT)
            print("\n".join(open(os.path.join(out, f"summary{pi}.txt")).read().splitlines()[:30]), flush=True)
            for p in dbs:
                os.remove(p)
    return 0


def _table(results: dict, benches: list[str], names: list[str], path: str) -> None:
    """Median samples/s per (config, arm), and each arm's delta against the first arm."""
    import statistics
    rows = [f"{'config':<70s} " + " ".join(f"{n:>16s}" for n in names)]
    for bi, bargs in enumerate(benches):
        med = {n: statistics.median(v) for n, v in results.get(bi, {}).items()}
        base = med.get(names[0])
        cells = []
        for n in names:
            if n not in med:
                cells.append(f"{'-':>16s}")
            elif n == names[0] or not base:
                cells.append(f"{med[n]:>16.2f}")
            else:
                cells.append(f"{med[n]:>8.2f} {100 * (med[n] / base - 1):+6.2f}%")
        rows.append(f"{bargs[:70]:<70s} " + " ".join(cells))
    txt = "\n".join(rows)
    with open(path, "w") as f:
        f.write(txt + "\n")
    print(txt, flush=True)


def _prof_steps(args: str) -> int:
    """Steps a profiled eager bench run executes (warmup + timed)."""
    t = shlex.split(args)
    get = lambda k, dflt: int(t[t.index(k) + 1]) if k in t else dflt  # noqa: E731
    return get("--steps", 20) + get("--warmup", 5)


if __name__ == "__main__":
    sys.exit(main())
