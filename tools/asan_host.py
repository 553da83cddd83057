"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the native runtime.

GPU sanitizers are not available on the MI355X pool, so this instruments the HOST C++ of the extension — the
native gradient reducer (csrc/reducer.cpp: bucket state machine, readiness bookkeeping, c10d launches, hook
lifetime) and the torch/pybind glue with its shape / pointer validation (csrc/bind.cpp) — and runs the
multi-rank CPU tests (gloo, 2-4 ranks) that drive them, in this container, without a GPU:

  1. csrc/*.cpp -> g++ -fsanitize=address,undefined -fno-omit-frame-pointer -O1 -g;
  2. linked with the normal (uninstrumented) HIP kernel objects of build/native/ into build/asan/_C*.so;
  3. pytest with LD_PRELOAD=libasan (+ libstdc++), DLLM_NATIVE_SO pointing at that library (distributed_llms_example_amd/_ext.py)
     and UBSAN_OPTIONS=halt_on_error=1: any heap overflow, use-after-free or UB report fails the run.

    python tools/asan_host.py [-k PYTEST_EXPR] [--out profiles/r2_asan_host.txt]
"""
from __future__ import annotations

import argparse
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import build_native  # noqa: E402

OUT_DIR = os.path.join(ROOT, "build", "asan")
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
DEFAULT_K = "reducer or bucket or collective or no_sync or grad_accumulation or train_task or accelerator"


def build() -> str:
    build_native.build(verbose=False)  # the HIP objects (uninstrumented device + host launch code)
    os.makedirs(OUT_DIR, exist_ok=True)
    inc, lib, abi = build_native._torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    objs = sorted(glob.glob(os.path.join(build_native.BUILD, "*.hip.o")))
    for src in sorted(glob.glob(os.path.join(build_native.CSRC, "*.cpp"))):
        obj = os.path.join(OUT_DIR, os.path.basename(src) + ".o")
        cmd = ["g++", "-O1", "-g", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
               "-D__HIP_PLATFORM_AMD__=1", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
               "-DUSE_C10D_GLOO", "-DUSE_C10D_NCCL", "-DUSE_DISTRIBUTED", "-Wno-deprecated-declarations",
               "-I", build_native.CSRC, "-I", py_inc] + SAN
        for i in inc:
            cmd += ["-I", i]
        build_native._run(cmd + ["-c", src, "-o", obj])
        objs.append(obj)
    so = os.path.join(OUT_DIR, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))
    build_native._run(["g++", "-shared", "-fPIC", "-o", so] + objs + SAN + [
        f"-L{lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
        "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}", "-Wl,-rpath,/opt/rocm/lib"])
    return so


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-k", default=DEFAULT_K)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    so = build()
    lib = lambda n: subprocess.run(["g++", f"-print-file-name={n}"], capture_output=True, text=True).stdout.strip()
    # libstdc++ right after the ASAN runtime: otherwise its __cxa_throw interceptor finds no real symbol and aborts on
    # the first C++ exception (torch's collective-mismatch errors are exceptions)
    env = dict(os.environ, LD_PRELOAD=f"{lib('libasan.so')} {lib('libstdc++.so')}", DLLM_NATIVE_SO=so,
               # torch's own (uninstrumented) allocations: no leak report; ODR / new-delete checks concern torch
               ASAN_OPTIONS="detect_leaks=0:new_delete_type_mismatch=0:alloc_dealloc_mismatch=0:"
                            "detect_odr_violation=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    cmd = [sys.executable, "-m", "pytest", "tests", "-m", "not gpu", "-q", "-x", "-p", "no:cacheprovider",
           "-k", a.k, "-p", "no:xdist"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True)
    log = r.stdout + r.stderr
    probe = subprocess.run([sys.executable, "-c", "from distributed_llms_example_amd import _ext; "
                            "print(_ext.native().__file__)"], env=env, cwd=ROOT, capture_output=True, text=True)
    report = (f"# host ASAN+UBSan run (tools/asan_host.py): {' '.join(SAN)}\n# library: {probe.stdout.strip()}\n"
              f"# pytest -k '{a.k}' -> exit {r.returncode}\n" + "\n".join(log.strip().splitlines()[-15:]) + "\n")
    sanitizer_hits = [l for l in log.splitlines() if "ERROR: AddressSanitizer" in l or "runtime error:" in l]
    report += f"# sanitizer reports: {len(sanitizer_hits)}\n" + "\n".join(sanitizer_hits[:20])
    print(report)
    if a.out:
        with open(a.out, "w") as f:
            f.write(report + "\n")
    return 0 if r.returncode == 0 and not sanitizer_hits else 1


if __name__ == "__main__":
    sys.exit(main())
