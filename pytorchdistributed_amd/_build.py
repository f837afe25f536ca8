"""In-tree native build of ``pytorchdistributed_amd._C`` (HIP kernels for gfx950 + C++ runtime).

No hipify, no ``torch.utils.cpp_extension`` JIT cache: a ninja file is generated next to the sources
and the resulting ``_C*.so`` is written into the package directory, so the snapshot ``gpurun`` ships
to the MI355X box already carries the compiled extension.

* ``csrc/kernels/*.hip``  -> ``hipcc --offload-arch=gfx950`` (pure HIP, no torch headers: fast)
* ``csrc/runtime/*.cpp``  -> host C++ (pybind11 only)
* ``csrc/comm/*.cpp``     -> host C++ against HIP + RCCL (torch's bundled librccl, one RCCL per process)
* ``csrc/bindings.cpp``   -> host C++ against the torch headers
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pytorchdistributed_amd")
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PDA_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_C"


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def so_path() -> str:
    return os.path.join(PKG, EXT_NAME + _ext_suffix())


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _sources():
    hip = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    rt = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    comm = sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    return hip, rt, comm, [os.path.join(CSRC, "bindings.cpp")]


def write_ninja(debug: bool = False) -> str:
    import pybind11

    tinc, tlib, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    os.makedirs(BUILD, exist_ok=True)
    hip, rt, comm, bind = _sources()
    opt = "-O0 -g" if debug else "-O3"
    common_inc = f"-I{CSRC}/include -I{CSRC}/runtime"
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    cxx = os.environ.get("CXX", "g++")
    lines = [
        "ninja_required_version = 1.3",
        f"hipcc = {hipcc}",
        f"cxx = {cxx}",
        f"hipflags = --offload-arch={ARCH} {opt} -std=c++17 -fPIC -Wall -Wno-unused-function {common_inc}",
        f"rtflags = {opt} -std=c++17 -fPIC -Wall {common_inc} -I{pybind11.get_include()} -I{pyinc}"
        f" -D_GLIBCXX_USE_CXX11_ABI={abi}",
        f"commflags = {opt} -std=c++17 -fPIC -Wall {common_inc} -I{pybind11.get_include()} -I{pyinc}"
        f" -isystem {ROCM}/include -D__HIP_PLATFORM_AMD__=1 -D_GLIBCXX_USE_CXX11_ABI={abi}",
        f"bindflags = -O2 -std=c++17 -fPIC {common_inc} -I{pybind11.get_include()} -I{pyinc} "
        + " ".join(f"-isystem {p}" for p in tinc)
        + f" -isystem {ROCM}/include -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_EXTENSION_NAME={EXT_NAME}"
        f" -DTORCH_API_INCLUDE_EXTENSION_H -D_GLIBCXX_USE_CXX11_ABI={abi}",
        f"ldflags = -shared -fPIC --offload-arch={ARCH} -L{tlib} -Wl,-rpath,{tlib} -lc10 -lc10_hip -ltorch -ltorch_cpu"
        f" -ltorch_hip -ltorch_python -lrccl -L{ROCM}/lib -lamdhip64",
        "rule hip",
        "  command = $hipcc $hipflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIP $in",
        "rule rt",
        "  command = $cxx $rtflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule comm",
        "  command = $cxx $commflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX(rccl) $in",
        "rule bind",
        "  command = $cxx $bindflags -MD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX(torch) $in",
        "rule link",
        "  command = $hipcc $in -o $out $ldflags",
        "  description = LINK $out",
    ]
    objs = []
    for src, rule in ([(s, "hip") for s in hip] + [(s, "rt") for s in rt] + [(s, "comm") for s in comm]
                      + [(s, "bind") for s in bind]):
        rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
        obj = os.path.join(BUILD, rel + ".o")
        objs.append(obj)
        lines.append(f"build {obj}: {rule} {src}")
    lines.append(f"build {so_path()}: link " + " ".join(objs))
    lines.append(f"default {so_path()}")
    path = os.path.join(BUILD, "build.ninja")
    text = "\n".join(lines) + "\n"
    old = open(path).read() if os.path.exists(path) else None
    if old != text:
        with open(path, "w") as f:
            f.write(text)
    return path


def build(verbose: bool = False, jobs: int | None = None, debug: bool = False) -> str:
    """Compile every HIP/C++ source for gfx950 and link ``pytorchdistributed_amd/_C*.so``."""
    path = write_ninja(debug=debug)
    ninja = shutil.which("ninja")
    if ninja is None:
        import ninja as _ninja_mod  # the pip package ships the binary

        ninja = os.path.join(_ninja_mod.BIN_DIR, "ninja")
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = [ninja, "-C", BUILD, "-f", path, f"-j{jobs}"]
    if verbose:
        cmd.append("-v")
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        sys.stderr.write(res.stdout)
        raise RuntimeError("native build of pytorchdistributed_amd._C failed")
    if verbose:
        print(res.stdout)
    return so_path()


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, debug="--debug" in sys.argv))
