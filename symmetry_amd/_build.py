"""In-tree native build for symmetry_amd.

Two native artefacts are produced, both next to the Python sources so they
travel with the repo snapshot to the GPU box:

* ``symmetry_amd/_C.so`` -- the CDNA4 (gfx950) HIP kernels plus the
  ``TORCH_LIBRARY(symmetry_amd, ...)`` op registrations.  Kernel TUs
  (``csrc/kernels/*.hip``) are compiled with ``hipcc --offload-arch=gfx950``
  WITHOUT torch headers (fast); only ``csrc/bindings/torch_ops.cpp`` sees the
  ATen headers.  No hipify step, no CUDA sources: the kernels are HIP written
  for CDNA4 directly.
* ``symmetry_amd/runtime/_runtime.so`` -- native runtime pieces around the
  GPU path (``csrc/runtime``): the shared-memory step-metadata ring that
  drives tensor-parallel workers (R4).
* ``symmetry_amd/net/_native.so`` -- the C++ P2P plane (crypto over OpenSSL
  libcrypto, Noise XX, secretstream framing, epoll transport), the
  MI355X-box equivalent of the reference's native deps sodium-native and
  udx-native (``package-lock.json:5725``, ``:6241``).

The build is incremental (mtime based) and parallel.  ``python -m
symmetry_amd._build`` builds everything; ``__graft_entry__.build()`` calls
:func:`build_all`.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "symmetry_amd")
CSRC = os.path.join(ROOT, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")

ARCH = os.environ.get("SYMMETRY_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

KERNEL_SO = os.path.join(PKG, "_C.so")
NET_SO = os.path.join(PKG, "net", "_native.so")
RUNTIME_SO = os.path.join(PKG, "runtime", "_runtime.so")


def _torch_paths():
    import torch  # noqa: WPS433 (build-time only)

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd, verbose: bool):
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"build step failed ({res.returncode}):\n{' '.join(cmd)}\n{res.stdout}")
    if verbose and res.stdout.strip():
        print(res.stdout, flush=True)


def _jobs() -> int:
    env = os.environ.get("MAX_JOBS")
    if env and env.isdigit():
        return max(1, min(16, int(env)))
    return max(1, min(8, os.cpu_count() or 1))


# --------------------------------------------------------------------------------------
# HIP kernels + torch op bindings
# --------------------------------------------------------------------------------------
HIP_FLAGS = [
    "-O3",
    "-std=c++17",
    "-fPIC",
    f"--offload-arch={ARCH}",
    "-ffp-contract=fast",
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
]


def build_kernels(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    kdir = os.path.join(CSRC, "kernels")
    headers = glob.glob(os.path.join(kdir, "*.h")) + glob.glob(os.path.join(kdir, "*.cuh"))
    sources = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    tinc, tlib, abi = _torch_paths()
    jobs = []
    objs = []
    for src in sources:
        obj = os.path.join(OBJ, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            cmd = [HIPCC, "-c", src, "-o", obj, "-I", kdir] + HIP_FLAGS
            jobs.append(cmd)
    for bsrc in sorted(glob.glob(os.path.join(CSRC, "bindings", "*.cpp"))):
        bobj = os.path.join(OBJ, "bind_" + os.path.basename(bsrc) + ".o")
        objs.append(bobj)
        if force or _newer(bobj, [bsrc] + headers):
            cmd = [HIPCC, "-c", bsrc, "-o", bobj, "-I", kdir, "-O2", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
                   "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                   "-DTORCH_EXTENSION_NAME=_C", "-Wno-unused-result", "-Wno-deprecated-declarations"]
            for i in tinc:
                cmd += ["-isystem", i]
            jobs.append(cmd)
    if jobs:
        with cf.ThreadPoolExecutor(_jobs()) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or jobs or _newer(KERNEL_SO, objs):
        cmd = [HIPCC, "-shared", "-o", KERNEL_SO] + objs + [
            f"--offload-arch={ARCH}", "-L", tlib, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch",
            "-lrccl",
            f"-Wl,-rpath,{tlib}",
        ]
        _run(cmd, verbose)
    return KERNEL_SO


# --------------------------------------------------------------------------------------
# C++ network plane (pybind11 module)
# --------------------------------------------------------------------------------------
def build_net(verbose: bool = False, force: bool = False) -> str:
    import pybind11

    os.makedirs(OBJ, exist_ok=True)
    ndir = os.path.join(CSRC, "net")
    headers = glob.glob(os.path.join(ndir, "*.h"))
    sources = sorted(s for s in glob.glob(os.path.join(ndir, "*.cpp")) if not s.endswith("selftest.cpp"))
    pyinc = sysconfig.get_paths()["include"]
    cxx = shutil.which("g++") or "c++"
    flags = ["-O2", "-g", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-fvisibility=hidden"]
    extra = os.environ.get("SYMMETRY_AMD_NET_CXXFLAGS", "").split()
    jobs, objs = [], []
    for src in sources:
        obj = os.path.join(OBJ, "net_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs.append([cxx, "-c", src, "-o", obj, "-I", ndir, "-I", pybind11.get_include(), "-I", pyinc]
                        + flags + extra)
    if jobs:
        with cf.ThreadPoolExecutor(_jobs()) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs))
    if force or jobs or _newer(NET_SO, objs):
        _run([cxx, "-shared", "-o", NET_SO] + objs + ["-lcrypto", "-lpthread"] + extra, verbose)
    return NET_SO


def build_runtime(verbose: bool = False, force: bool = False) -> str:
    """csrc/runtime/*.cpp -> symmetry_amd/runtime/_runtime.so (pybind11, host C++ only)."""
    import pybind11

    os.makedirs(OBJ, exist_ok=True)
    rdir = os.path.join(CSRC, "runtime")
    sources = sorted(glob.glob(os.path.join(rdir, "*.cpp")))
    headers = glob.glob(os.path.join(rdir, "*.h"))
    pyinc = sysconfig.get_paths()["include"]
    cxx = shutil.which("g++") or "c++"
    flags = ["-O2", "-g", "-std=c++17", "-fPIC", "-Wall", "-fvisibility=hidden"]
    extra = os.environ.get("SYMMETRY_AMD_RUNTIME_CXXFLAGS", "").split()
    jobs, objs = [], []
    for src in sources:
        obj = os.path.join(OBJ, "rt_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            jobs.append([cxx, "-c", src, "-o", obj, "-I", rdir, "-I", pybind11.get_include(), "-I", pyinc]
                        + flags + extra)
    for c in jobs:
        _run(c, verbose)
    if force or jobs or _newer(RUNTIME_SO, objs):
        _run([cxx, "-shared", "-o", RUNTIME_SO] + objs + ["-lrt", "-lpthread"] + extra, verbose)
    return RUNTIME_SO


SELFTEST = os.path.join(ROOT, "build", "net_selftest_asan")


def build_selftest(verbose: bool = False, force: bool = False) -> str:
    """Host-only AddressSanitizer + UBSan build of the P2P plane and its self-test driver
    (csrc/net/selftest.cpp).  GPU sanitizers are not used: this is CPU code."""
    ndir = os.path.join(CSRC, "net")
    srcs = [os.path.join(ndir, f) for f in ("crypto.cpp", "noise.cpp", "transport.cpp", "selftest.cpp")]
    headers = glob.glob(os.path.join(ndir, "*.h"))
    os.makedirs(os.path.dirname(SELFTEST), exist_ok=True)
    if force or _newer(SELFTEST, srcs + headers):
        cxx = shutil.which("g++") or "c++"
        _run([cxx, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
              "-fno-sanitize-recover=undefined", "-I", ndir] + srcs + ["-o", SELFTEST, "-lcrypto", "-lpthread"],
             verbose)
    return SELFTEST


def build_all(verbose: bool = False, force: bool = False):
    net = build_net(verbose, force)
    build_runtime(verbose, force)
    ker = build_kernels(verbose, force)
    return ker, net


if __name__ == "__main__":
    force = "--force" in sys.argv
    verbose = "-v" in sys.argv or "--verbose" in sys.argv
    what = [a for a in sys.argv[1:] if not a.startswith("-")]
    if not what or "net" in what:
        print(build_net(verbose, force))
    if not what or "kernels" in what:
        print(build_kernels(verbose, force))
    if not what or "runtime" in what:
        print(build_runtime(verbose, force))
    if "selftest" in what:
        print(build_selftest(verbose, force))
