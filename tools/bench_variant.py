#!/usr/bin/env python
"""bench.py with HipEncoder variant attributes overridden (A/B of fused kernels against the
per-layer path on the whole training loop; diagnostics, not the headline).

    python tools/bench_variant.py fused_pool_wgrad0=0 fused_pool_conv_bwd=0 -- --steps 20
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    sets = dict(kv.split("=") for kv in argv[:cut])
    from microbeast_amd.ops import encoder as E
    init = E.HipEncoder.__init__

    def patched(self, *a, **k):
        init(self, *a, **k)
        for key, v in sets.items():
            assert hasattr(self, key), key
            setattr(self, key, bool(int(v)))
    E.HipEncoder.__init__ = patched
    import bench
    return bench.main(argv[cut + 1:])


if __name__ == "__main__":
    sys.exit(main())
