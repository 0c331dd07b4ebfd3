#!/usr/bin/env python
"""bench.py with HipEncoder variant attributes overridden (A/B of fused kernels against the
per-layer path on the whole training loop; diagnostics, not the headline).

    python tools/bench_variant.py fused_pool_wgrad0=0 fused_pool_conv_bwd=0 -- --steps 20
    python tools/bench_variant.py rt.fused_act=0 fused_tail=0 -- --steps 20   (graph step,
        per-stage inference kernels)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    sets = dict(kv.split("=") for kv in argv[:cut])
    lib = sets.pop("lib", None)  # lib=variants/<name>: a tools/variant.py build of the kernels
    if lib:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from variant import use_lib
        use_lib(lib)
    rt_sets = {k[3:]: v for k, v in sets.items() if k.startswith("rt.")}
    nat_sets = {k[7:]: v for k, v in sets.items() if k.startswith("native.")}
    sets = {k: v for k, v in sets.items() if not k.startswith(("rt.", "native."))}
    if nat_sets:  # kernel-library setters, e.g. native.mbk_set_work_queues=0 or
        from microbeast_amd import _native as N  # native.mbk_set_work_queue_site=5:0
        for key, v in nat_sets.items():
            N.check(getattr(N.kernels(), key)(*[int(x) for x in v.split(":")]), key)
    if rt_sets:  # GpuActorRuntime keyword overrides, e.g. rt.fused_act=0 (the graph step)
        from microbeast_amd.runtime import gpu_actors as G
        rinit = G.GpuActorRuntime.__init__

        def rpatched(self, *a, **k):
            for key, v in rt_sets.items():
                k[key] = int(v)
            rinit(self, *a, **k)
        G.GpuActorRuntime.__init__ = rpatched
    from microbeast_amd.ops import encoder as E
    init = E.HipEncoder.__init__

    def patched(self, *a, **k):
        init(self, *a, **k)
        for key, v in sets.items():
            assert hasattr(self, key), key
            setattr(self, key, bool(int(v)))
    E.HipEncoder.__init__ = patched
    import bench
    return bench.main([x for x in argv[cut + 1:] if x != "--"])  # (a second "--" from wrappers)


if __name__ == "__main__":
    sys.exit(main())
