#!/usr/bin/env python3
"""Build the native extension ``distributed-deep-learning_amd/_C.so`` for gfx950.

* ``csrc/kernels/*.hip``  -> hipcc --offload-arch=gfx950 (device + host launchers)
* ``csrc/runtime/*.cpp``  -> g++ (shared-memory mailbox; no HIP)
* ``csrc/bindings.cpp``   -> g++ against the torch / pybind11 headers
* link                    -> hipcc -shared, rpath to torch's libs

Plain hipcc/g++ invocations (no hipify, no JIT cache): the ``.so`` lands in-tree so it
ships to the GPU box with the repo snapshot.  Objects are rebuilt only when a source or
header is newer.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "distributed-deep-learning_amd")
CSRC = os.path.join(PKG, "csrc")
# DDL_BUILD_TAG=x: a side build (objects in _build_x/, extension _C_x.so) with the compile-time
# knobs of DDL_EXTRA_CFLAGS, loaded at run time with DDL_SO=_C_x.so (same-box A/B)
_TAG = os.environ.get("DDL_BUILD_TAG", "")
BUILD = os.path.join(PKG, "_build" + (f"_{_TAG}" if _TAG else ""))
OUT = os.path.join(PKG, f"_C_{_TAG}.so" if _TAG else "_C.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension
    inc = cpp_extension.include_paths(device_type="cuda") if "device_type" in \
        cpp_extension.include_paths.__code__.co_varnames else cpp_extension.include_paths(True)
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(src_files, obj):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {os.path.basename(cmd[-1])}")
    return r


def build(verbose: bool = False, jobs: int | None = None) -> str:
    os.makedirs(BUILD, exist_ok=True)
    inc, tlib, abi = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    bind = os.path.join(CSRC, "bindings.cpp")
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
              *os.environ.get("DDL_EXTRA_CFLAGS", "").split()]
    steps = []
    objs = []
    for s in hip_srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer([s] + headers, o):
            steps.append([HIPCC, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common,
                          "-c", "-o", o, s])
    for s in cpp_srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer([s] + headers, o):
            steps.append(["g++", *common, "-c", "-o", o, s])
    ob = os.path.join(BUILD, "bindings.cpp.o")
    objs.append(ob)
    if _newer([bind] + headers, ob):
        steps.append(["g++", *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                      "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
                      f"-I{ROCM}/include", f"-I{py_inc}", *[f"-I{p}" for p in inc],
                      "-Wno-deprecated-declarations", "-c", "-o", ob, bind])
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        for cmd in steps:
            if verbose:
                print(" ".join(cmd))
        list(ex.map(_run, steps))
    if steps or not os.path.exists(OUT):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT, *objs,
                f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                "-ltorch_python", "-ldl", f"-Wl,-rpath,{tlib}", "-lrt"]
        if verbose:
            print(" ".join(link))
        _run(link)
    return OUT


if __name__ == "__main__":
    t = build(verbose="-v" in sys.argv)
    print("built", t)
