"""Build libmcroute.so (HIP, gfx950) in-tree.

The library is compiled with ``hipcc --offload-arch=gfx950`` directly from ``csrc/``; the result
lands next to this file (``lib/libmcroute.so``) so it travels with the repository snapshot.
``-ffp-contract=off`` is load-bearing: the routing arithmetic must keep separate multiply and add
roundings to match the reference bit for bit.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC_DIR = os.path.join(os.path.dirname(PKG_DIR), "csrc")
REPO = os.path.dirname(os.path.dirname(PKG_DIR))
INCLUDE = os.path.join(REPO, "include")
LIB_DIR = os.path.join(PKG_DIR, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libmcroute.so")

ARCH = os.environ.get("MCROUTE_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libmcroute.so)")


def sources():
    return sorted(glob.glob(os.path.join(SRC_DIR, "*.cpp")) +
                  glob.glob(os.path.join(SRC_DIR, "*.hip")))


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = sources() + glob.glob(os.path.join(SRC_DIR, "*.hpp")) + \
        glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB_PATH
    os.makedirs(LIB_DIR, exist_ok=True)
    tmp = LIB_PATH + f".{os.getpid()}.tmp"
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-ffp-contract=off", "-fno-fast-math", "-Wall", "-Wno-unused-function",
           "-I", INCLUDE, "-I", SRC_DIR, "-o", tmp] + sources() + \
        ["-L/opt/rocm/lib", "-lrocsolver", "-lrocblas", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
