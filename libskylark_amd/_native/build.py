"""Build the native HIP/C++ library ``libskylark_hip.so`` for gfx950, in-tree.

Every ``src/*.hip`` / ``src/*.cpp`` file is compiled with ``hipcc
--offload-arch=gfx950`` into an object and linked into one shared library
next to this file (so it travels to the GPU box with the repository
snapshot).  Objects are rebuilt only when their source or any header
changed.  No hipify, no CUDA paths: the sources are written for CDNA4.

Usage:  python -m libskylark_amd._native.build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "src")
INC = os.path.join(HERE, "include")
OBJ = os.path.join(HERE, "build")
LIB = os.path.join(HERE, "libskylark_hip.so")
CAPI_SRC = os.path.join(HERE, "capi", "skylark_capi.cpp")
CAPI_LIB = os.path.join(HERE, "libskylark_capi.so")
ARCH = os.environ.get("SKH_GFX_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

COMMON_FLAGS = [
    "-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I", INC,
    "-fvisibility=hidden", "-Wno-unused-result", "-munsafe-fp-atomics",
    # zstd-compressed device code bundles (the HIP runtime inflates them at
    # load): the library's fat binary shrinks ~3.5x, and so does every push
    "--offload-compress",
]


def _sources():
    out = []
    for f in sorted(os.listdir(SRC)):
        if f.endswith((".hip", ".cpp")):
            out.append(os.path.join(SRC, f))
    return out


def _header_digest():
    h = hashlib.sha1()
    for f in sorted(os.listdir(INC)):
        with open(os.path.join(INC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _obj_path(src, hdr):
    with open(src, "rb") as fh:
        d = hashlib.sha1(fh.read() + hdr.encode() + " ".join(COMMON_FLAGS).encode()).hexdigest()[:12]
    base = os.path.splitext(os.path.basename(src))[0]
    return os.path.join(OBJ, f"{base}.{d}.o")


def _compile(src, obj):
    cmd = [HIPCC] + COMMON_FLAGS + ["-c", src, "-o", obj + ".tmp"]
    if src.endswith(".cpp"):
        cmd = [HIPCC] + COMMON_FLAGS + ["-x", "hip", "-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    hdr = _header_digest()
    srcs = _sources()
    objs = [_obj_path(s, hdr) for s in srcs]
    todo = [(s, o) for s, o in zip(srcs, objs) if force or not os.path.exists(o)]
    jobs = jobs or min(8, max(1, (os.cpu_count() or 2)))
    jobs = min(jobs, 16)
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, s, o) for s, o in todo]
            for f in futs:
                o = f.result()
                if verbose:
                    print("compiled", os.path.basename(o))
    need_link = force or bool(todo) or not os.path.exists(LIB)
    if not need_link:
        lib_m = os.path.getmtime(LIB)
        need_link = any(os.path.getmtime(o) > lib_m for o in objs)
    if need_link:
        tmp = LIB + f".{os.getpid()}.tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        os.replace(tmp, LIB)
        if verbose:
            print("linked", LIB)
    build_capi(force)
    # drop stale objects of older source versions
    keep = set(objs)
    for f in os.listdir(OBJ):
        p = os.path.join(OBJ, f)
        if f.endswith(".o") and p not in keep:
            try:
                os.remove(p)
            except OSError:
                pass
    return LIB


def build_capi(force: bool = False) -> str:
    """C API library (host C++; embeds/joins CPython for the runtime paths, loads
    libskylark_hip.so + rocBLAS for the DeviceMatrix paths; no device code)."""
    srcs = [CAPI_SRC, os.path.join(HERE, "capi", "native_sketch.hpp"), os.path.join(HERE, "capi", "native_device.hpp"),
            os.path.join(INC, "sl_rng.hpp"), os.path.join(INC, "sl_perm.hpp")]
    if not force and os.path.exists(CAPI_LIB) and all(os.path.getmtime(CAPI_LIB) >= os.path.getmtime(f) for f in srcs):
        return CAPI_LIB
    import sysconfig
    inc = sysconfig.get_paths()["include"]
    libdir = sysconfig.get_config_var("LIBDIR")
    ver = sysconfig.get_config_var("LDVERSION") or sysconfig.get_python_version()
    tmp = CAPI_LIB + f".{os.getpid()}.tmp"
    cmd = [os.environ.get("CXX", "g++"), "-O3", "-fPIC", "-shared", "-std=c++17", "-fvisibility=hidden",
           "-I", inc, "-I", INC, CAPI_SRC, "-o", tmp, f"-L{libdir}", f"-lpython{ver}", "-ldl", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"C API build failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, CAPI_LIB)
    return CAPI_LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args(argv)
    print(build(force=a.force, jobs=a.j, verbose=True))


if __name__ == "__main__":
    sys.exit(main())
