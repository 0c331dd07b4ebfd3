"""Every C entry point the ctypes layer declares (microbeast_amd/_native.py _SIGS) is exported
by the built kernel library: a launcher whose symbol went missing from a .hip edit fails here,
on the CPU, instead of on the GPU box."""
import subprocess
from pathlib import Path

import pytest

from microbeast_amd import _native as N

LIB = Path(N.__file__).resolve().parent / "_lib" / "libmbk_kernels.so"


@pytest.mark.skipif(not LIB.exists(), reason="kernel library not built (python __graft_entry__.py)")
def test_every_declared_kernel_entry_point_is_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB)], capture_output=True, text=True,
                         check=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    missing = sorted(k for k in N._SIGS if k.startswith("mbk_") and k not in syms)
    assert not missing, f"declared in _native._SIGS but not exported: {missing}"
