#!/usr/bin/env python
"""Build an A/B variant of the native libraries with extra ``-D`` defines for the kernel sources
into ``variants/<name>/`` (git-ignored, travels to the GPU box with the tree), for tools that take
``--lib variants/<name>`` (tools/act_phases.py).

    python tools/variant.py <name> -DMBK_HA_MB=2 [-DOTHER=1 ...]
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def use_lib(path: str | None) -> None:
    """Point microbeast_amd._native at a variant library directory (before the first load)."""
    if not path:
        return
    from pathlib import Path

    from microbeast_amd import _native as N
    assert N._kern is None, "use_lib must run before the kernel library is loaded"
    N._LIB = Path(path).resolve()


def main() -> None:
    name, defines = sys.argv[1], sys.argv[2:]
    assert all(d.startswith("-D") for d in defines), defines
    from microbeast_amd.csrc import build as b
    out = b.build(defines=defines, libdir=os.path.join(ROOT, "variants", name))
    print(out)


if __name__ == "__main__":
    main()
