"""Build the in-tree native extension ``distributed_llms_example_amd/_C*.so`` for gfx950.

No hipify, no CUDA compatibility layer: every ``csrc/*.hip`` file is plain HIP compiled by
``hipcc --offload-arch=gfx950`` into an object with C-ABI launchers; ``csrc/bind.cpp`` (torch +
pybind11 glue, host-only) is compiled by the host C++ compiler with torch's headers; both are linked
into one shared object next to the Python package so it travels with the repo snapshot.
Incremental by content: an object is rebuilt when the hash of its source, the headers or its command line changed
(``<obj>.sha256`` sidecars).  Every link writes the provenance record ``distributed_llms_example_amd/_C.build.json``
(arch, hipcc version, sha256 of every source and of the .so, objects rebuilt); ``_ext`` compares it with the sources
at import and refuses a stale library on the GPU.

    python tools/build_native.py [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import subprocess
import sys
import sysconfig
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
PKG = os.path.join(ROOT, "distributed_llms_example_amd")
ARCH = os.environ.get("DLLM_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


# Per-source flags.  attn.hip: no SLP vectorisation — packing independent f32 adds / FMAs into v_pk_* beside MFMAs
# costs more issue cycles than the scalar ops (MI355X_MICROARCH.md, per-instruction constants) and the compiler adds
# v_mov shuffles to form the register pairs.
EXTRA_FLAGS = {"attn.hip": ["-fno-slp-vectorize"]}
# DLLM_HIPFLAGS_EXTRA: extra flags for every HIP source (A/B builds of a kernel variant, e.g. "-DDKDV_PIPE=0"); part
# of the object key, so switching it back rebuilds the default objects
_ENV_FLAGS = os.environ.get("DLLM_HIPFLAGS_EXTRA", "").split()
_ENV_FLAGS_SRC = os.environ.get("DLLM_HIPFLAGS_EXTRA_SRC", "")  # only this source (default: every HIP source)


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def so_path() -> str:
    return os.path.join(PKG, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _sha(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _stale(obj: str, key: str) -> bool:
    """Rebuild decision by CONTENT: an object is current when its sidecar holds the hash of (source, every header,
    command line) it was built from — not by file times, which a checkout or copy can reorder."""
    side = obj + ".sha256"
    if not (os.path.exists(obj) and os.path.exists(side)):
        return True
    with open(side) as f:
        return f.read().strip() != key


def _key(src: str, headers, cmd) -> str:
    h = hashlib.sha256()
    for p in [src] + sorted(headers):
        h.update(os.path.basename(p).encode())
        h.update(_sha(p).encode())
    h.update(" ".join(c for c in cmd if c not in ("-o",) and not c.endswith(".o")).encode())
    return h.hexdigest()


def source_hashes() -> dict:
    """{file name: sha256} of every native source and header (the provenance record's and _ext's staleness check)."""
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")) +
                   glob.glob(os.path.join(CSRC, "*.h")))
    return {os.path.basename(p): _sha(p) for p in files}


def record_path() -> str:
    return os.path.join(PKG, "_C.build.json")


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    jobs_list = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        cmd = ([HIPCC, f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
                "-munsafe-fp-atomics"] + EXTRA_FLAGS.get(os.path.basename(src), [])
               + (_ENV_FLAGS if _ENV_FLAGS_SRC in ("", os.path.basename(src)) else [])
               + ["-I", CSRC, "-c", src, "-o", obj])
        key = _key(src, headers, cmd)
        if force or _stale(obj, key):
            jobs_list.append((cmd, obj, key))
    # host C++ (torch + pybind11 glue, native runtime pieces): every csrc/*.cpp
    for cpp_src in sorted(glob.glob(os.path.join(CSRC, "*.cpp"))):
        cpp_obj = os.path.join(BUILD, os.path.basename(cpp_src) + ".o")
        objs.append(cpp_obj)
        cmd = [CXX, "-O2", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
               "-D__HIP_PLATFORM_AMD__=1", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
               "-DUSE_C10D_GLOO", "-DUSE_C10D_NCCL", "-DUSE_DISTRIBUTED",
               "-Wno-deprecated-declarations", "-I", CSRC, "-I", py_inc]
        for i in inc:
            cmd += ["-I", i]
        cmd += ["-c", cpp_src, "-o", cpp_obj]
        key = _key(cpp_src, headers, cmd)
        if force or _stale(cpp_obj, key):
            jobs_list.append((cmd, cpp_obj, key))
    if jobs_list:
        def one(job):
            cmd, obj, key = job
            _run(cmd)
            with open(obj + ".sha256", "w") as f:
                f.write(key)
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            futs = [ex.submit(one, j) for j in jobs_list]
            for f in futs:
                f.result()
    out = so_path()
    srcs = source_hashes()
    rec = None
    if os.path.exists(record_path()):
        with open(record_path()) as f:
            rec = json.load(f)
    fresh = (rec is not None and rec.get("sources") == srcs and rec.get("arch") == ARCH and os.path.exists(out)
             and rec.get("so_sha256") == _sha(out))
    if force or jobs_list or not fresh:
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + [
            f"-L{lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
            "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}", "-Wl,-rpath,/opt/rocm/lib"]
        _run(link)
        rec = {"arch": ARCH, "hipcc": _run([HIPCC, "--version"]).splitlines()[0:2], "sources": srcs,
               "objects_rebuilt": [os.path.basename(j[1]) for j in jobs_list], "so": os.path.basename(out),
               "so_sha256": _sha(out), "built_at": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
        with open(record_path(), "w") as f:
            json.dump(rec, f, indent=1)
        if verbose:
            print(f"[build_native] linked {os.path.relpath(out, ROOT)} ({len(hip_srcs)} HIP sources, arch {ARCH}; "
                  f"{len(jobs_list)} objects rebuilt; provenance {os.path.relpath(record_path(), ROOT)})")
    elif verbose:
        print(f"[build_native] up to date: {os.path.relpath(out, ROOT)}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=8)
    a = ap.parse_args()
    build(force=a.force, jobs=a.j)


if __name__ == "__main__":
    sys.exit(main())
