"""Build libmcroute.so (HIP, gfx950) in-tree.

The library is compiled with ``hipcc --offload-arch=gfx950`` directly from ``csrc/``; the result
lands next to this file (``lib/libmcroute.so``) so it travels with the repository snapshot.
``-ffp-contract=off`` is load-bearing: the routing arithmetic must keep separate multiply and add
roundings to match the reference bit for bit.

Every source compiles to its own object (``lib/obj/``) in parallel; an object is rebuilt when
its source or any header is newer, then the objects are linked.  The library needs only the HIP
runtime (no rocBLAS / rocSOLVER: every dense kernel is the library's own).
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC_DIR = os.path.join(os.path.dirname(PKG_DIR), "csrc")
REPO = os.path.dirname(os.path.dirname(PKG_DIR))
INCLUDE = os.path.join(REPO, "include")
LIB_DIR = os.path.join(PKG_DIR, "lib")
OBJ_DIR = os.path.join(LIB_DIR, "obj")
LIB_PATH = os.path.join(LIB_DIR, "libmcroute.so")

ARCH = os.environ.get("MCROUTE_ARCH", "gfx950")
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-fno-fast-math", "-Wall", "-Wno-unused-function"]
LIBS = ["-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib", "-pthread"]
# host-only sources (*.cc: no device code) are built by the host C++ compiler
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libmcroute.so)")


def sources():
    return sorted(glob.glob(os.path.join(SRC_DIR, "*.cpp")) +
                  glob.glob(os.path.join(SRC_DIR, "*.hip")) +
                  glob.glob(os.path.join(SRC_DIR, "*.cc")))


def _cxx() -> str:
    for cand in (os.environ.get("CXX"), shutil.which("g++"), shutil.which("c++")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("no host C++ compiler (g++) found")


def _headers():
    return glob.glob(os.path.join(SRC_DIR, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def source_hash() -> str:
    """sha256 (first 16 hex digits) of every library source, header and the compile flags: the
    identity of a build.  Profiles measured on a build carry it (scripts/hbm_traffic.py) and
    bench.py reports a profile only for the build it was measured on."""
    import hashlib
    h = hashlib.sha256(" ".join(FLAGS + HOST_FLAGS).encode())
    for p in sorted(sources() + _headers()):
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _obj(src: str) -> str:
    return os.path.join(OBJ_DIR, os.path.basename(src) + ".o")


STAMP_PATH = LIB_PATH + ".stamp"


def _stale() -> bool:
    """The library is rebuilt when it is missing, when any source or header is newer, or when
    the build identity changed (a source added or deleted, other flags): the stamp written next
    to it holds the source_hash() it was built from."""
    if not os.path.exists(LIB_PATH) or not os.path.exists(STAMP_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    if any(os.path.getmtime(p) > t for p in sources() + _headers()):
        return True
    with open(STAMP_PATH) as f:
        return f.read().strip() != source_hash()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB_PATH
    os.makedirs(OBJ_DIR, exist_ok=True)
    hipcc = _hipcc()
    t_hdr = max((os.path.getmtime(p) for p in _headers()), default=0.0)

    def compile_one(src):
        obj = _obj(src)
        if (not force and os.path.exists(obj) and
                os.path.getmtime(obj) >= max(os.path.getmtime(src), t_hdr)):
            return
        tmp = obj + f".{os.getpid()}.tmp"
        if src.endswith(".cc"):
            cmd = [_cxx()] + HOST_FLAGS + ["-I", INCLUDE, "-I", SRC_DIR, "-c", "-o", tmp, src]
        else:
            cmd = [hipcc] + FLAGS + ["-I", INCLUDE, "-I", SRC_DIR, "-c", "-o", tmp, src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        os.replace(tmp, obj)

    srcs = sources()
    with ThreadPoolExecutor(max_workers=min(len(srcs), 6)) as ex:
        list(ex.map(compile_one, srcs))
    tmp = LIB_PATH + f".{os.getpid()}.tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + \
        [_obj(s) for s in srcs] + LIBS
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB_PATH)
    with open(STAMP_PATH, "w") as f:
        f.write(source_hash() + "\n")
    return LIB_PATH


def build_variant(name: str, extra_flags, verbose: bool = False) -> str:
    """Diagnostic / A-B build of the whole library with extra compile flags (e.g. a -D switch
    switch) into lib/exp/lib_<name>.so; bench.py / tests load it with MCROUTE_LIB=<path>."""
    out_dir = os.path.join(LIB_DIR, "exp")
    obj_dir = os.path.join(out_dir, "obj_" + name)
    os.makedirs(obj_dir, exist_ok=True)
    hipcc = _hipcc()
    extra = list(extra_flags)

    def compile_one(src):
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if src.endswith(".cc"):
            cmd = [_cxx()] + HOST_FLAGS + extra + ["-I", INCLUDE, "-I", SRC_DIR, "-c", "-o",
                                                     obj, src]
        else:
            cmd = [hipcc] + FLAGS + extra + ["-I", INCLUDE, "-I", SRC_DIR, "-c", "-o", obj,
                                             src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        return obj

    srcs = sources()
    with ThreadPoolExecutor(max_workers=min(len(srcs), 6)) as ex:
        objs = list(ex.map(compile_one, srcs))
    path = os.path.join(out_dir, f"lib_{name}.so")
    subprocess.check_call([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", path] +
                          objs + LIBS)
    return path


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--variant":
        # python _build.py --variant NAME [-DFLAG ...]
        print(build_variant(sys.argv[2], sys.argv[3:], verbose=True))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
