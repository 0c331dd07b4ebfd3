"""Native build driver for microbeast_amd (no hipify, no torch JIT).

Produces, in-tree under ``microbeast_amd/_lib/``:

* ``libmbk_kernels.so`` — every ``csrc/kernels/*.hip`` compiled by ``hipcc
  --offload-arch=gfx950`` (CDNA4 only) behind a plain C ABI (``mbk_api.h``),
  called from Python through ctypes with torch tensors' device pointers and
  the current HIP stream (so calls are hipGraph-capturable).
* ``_mbrt<ext>`` — the pybind11 runtime module: synthetic microRTS simulator,
  vectorised env, shared-memory index rings / seqlock, and the GPU actor
  engine (env worker threads + HIP driver thread). Host C++ (g++), links HIP
  runtime and ``libmbk_kernels.so``.

Objects are cached by a content hash of the source, its local headers and
the flags, so a rebuild after a one-file edit recompiles one file.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
LIBDIR = PKG / "_lib"
BUILD = PKG.parent / "build" / "native"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
ARCH = "gfx950"  # MI355X (CDNA4) only

KERNEL_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
    "-Wno-unused-variable", "-munsafe-fp-atomics", f"-I{HERE / 'include'}",
]
HOST_FLAGS = [
    "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-D__HIP_PLATFORM_AMD__",
    f"-I{ROCM / 'include'}", f"-I{HERE / 'include'}", "-pthread",
]


def _hipcc() -> str:
    p = ROCM / "bin" / "hipcc"
    if p.exists():
        return str(p)
    found = shutil.which("hipcc")
    if not found:
        raise RuntimeError("hipcc not found (ROCm required to build microbeast_amd kernels)")
    return found


def _digest(src: Path, flags: list[str]) -> str:
    h = hashlib.sha1()
    h.update(" ".join(flags).encode())
    h.update(src.read_bytes())
    for d in (HERE / "include", HERE / "kernels", HERE / "runtime", HERE / "env"):
        for f in sorted(d.glob("*.h")):
            h.update(f.name.encode())
            h.update(f.read_bytes())
    return h.hexdigest()


def _compile(cc: str, src: Path, flags: list[str], verbose: bool) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    dig = _digest(src, [cc] + flags)
    obj = BUILD / f"{src.stem}.{src.suffix[1:]}.{dig[:12]}.o"
    if obj.exists():
        return obj
    cmd = [cc, *flags, "-c", str(src), "-o", str(obj) + ".tmp"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(str(obj) + ".tmp", obj)
    return obj


def _link(cc: str, objs: list[Path], out: Path, extra: list[str], verbose: bool) -> None:
    out.parent.mkdir(parents=True, exist_ok=True)
    tmp = out.with_suffix(out.suffix + ".tmp")
    cmd = [cc, "-shared", "-o", str(tmp), *map(str, objs), *extra]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed: {out}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)


def kernel_sources() -> list[Path]:
    return sorted((HERE / "kernels").glob("*.hip"))


def runtime_sources() -> list[Path]:
    return sorted((HERE / "runtime").glob("*.cpp")) + sorted((HERE / "env").glob("*.cpp"))


def ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def build(verbose: bool = False, jobs: int | None = None, defines: list[str] | None = None,
          libdir: Path | None = None) -> dict:
    """Compile and link both libraries into ``libdir`` (default: the package's ``_lib``).
    ``defines`` (``-DNAME=V`` flags for the kernel sources) build an A/B variant of the kernel
    library, e.g. ``tools/variant.py``; the package itself always loads ``_lib``."""
    hipcc = _hipcc()
    libdir = Path(libdir) if libdir is not None else LIBDIR
    kflags = KERNEL_FLAGS + list(defines or [])
    cxx = os.environ.get("CXX", "g++")
    import pybind11  # noqa: WPS433 (build-time only)

    py_inc = sysconfig.get_paths()["include"]
    host_flags = HOST_FLAGS + [f"-I{py_inc}", f"-I{pybind11.get_include()}"]
    jobs = jobs or min(16, os.cpu_count() or 4)
    ks, rs = kernel_sources(), runtime_sources()
    with cf.ThreadPoolExecutor(jobs) as ex:
        kfut = [ex.submit(_compile, hipcc, s, kflags, verbose) for s in ks]
        rfut = [ex.submit(_compile, cxx, s, host_flags, verbose) for s in rs]
        kobj = [f.result() for f in kfut]
        robj = [f.result() for f in rfut]
    klib = libdir / "libmbk_kernels.so"
    _link(hipcc, kobj, klib, [f"--offload-arch={ARCH}", "-fPIC"], verbose)
    rt = libdir / f"_mbrt{ext_suffix()}"
    _link(cxx, robj, rt,
          [f"-L{libdir}", "-lmbk_kernels", f"-L{ROCM / 'lib'}", "-lamdhip64", "-pthread",
           "-Wl,-rpath,$ORIGIN"], verbose)
    return {"kernels": str(klib), "runtime": str(rt)}


if __name__ == "__main__":
    out = build(verbose="-v" in sys.argv)
    print(out)
