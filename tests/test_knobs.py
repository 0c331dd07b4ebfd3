"""The framework's environment switches are few, named, and documented.

Every ``MBK_*`` variable the package, bench.py or the native sources read must be one of
``KNOBS`` and appear in docs/DESIGN.md §12 ("Environment switches"); measured-and-rejected
kernel / engine variants are deleted, not left behind a switch (their numbers live in
DESIGN.md §9c). Each knob's behaviour is pinned below or where it acts:

* MBK_DIST_BACKEND, MBK_FORCE_PG -- test_force_pg_gloo_world1 (here); the RCCL side in
  tests/test_gpu_dist_rccl.py
* MBK_RCCL_HIGH_PRIORITY -- the RCCL group options (tests/test_gpu_dist_rccl.py builds it)
* MBK_NUMA_PIN -- test_numa_pin_off_keeps_affinity (here)
* MBK_REBUILD -- forces build.py on import (the build itself: __graft_entry__.build)
* MBK_STEP_TIMING, MBK_HB_STAMPS -- diagnostics only (timing splits / phase stamps on
  stderr and in the bench JSON); test_step_timing_is_diagnostic_only (here)
"""
import os
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]

KNOBS = {
    "MBK_DIST_BACKEND",        # gloo instead of RCCL (several ranks on one GPU, CPU tests)
    "MBK_FORCE_PG",            # a real process group at world size 1 (the RCCL path on 1 GPU)
    "MBK_RCCL_HIGH_PRIORITY",  # RCCL's internal stream at high priority (default on)
    "MBK_NUMA_PIN",            # per-rank NUMA / CPU pinning (default on)
    "MBK_REBUILD",             # rebuild the native libraries on import
    "MBK_STEP_TIMING",         # engine: HIP-event split of each policy step (diagnostics)
    "MBK_HB_STAMPS",           # head_bwd2: per-phase clock stamps on stderr (diagnostics)
}

_READ = re.compile(r"""(?:getenv|environ\.get|environ\[|environ\.setdefault)\(?\s*["'](MBK_[A-Z0-9_]+)""")


def _sources():
    for sub in ("microbeast_amd",):
        for p in (ROOT / sub).rglob("*"):
            if p.suffix in (".py", ".cpp", ".h", ".hip") and "__pycache__" not in p.parts:
                yield p
    for name in ("bench.py", "__graft_entry__.py"):
        yield ROOT / name


def test_env_switches_are_the_documented_few():
    read = {}
    for p in _sources():
        for m in _READ.finditer(p.read_text(errors="replace")):
            read.setdefault(m.group(1), []).append(str(p.relative_to(ROOT)))
    unknown = {k: v for k, v in read.items() if k not in KNOBS}
    assert not unknown, f"undocumented MBK_* switches: {unknown}"
    design = (ROOT / "docs" / "DESIGN.md").read_text()
    sec = design[design.index("## 12. Environment switches"):]
    for k in KNOBS:
        assert k in sec, f"{k} missing from DESIGN.md §12"
    assert len(KNOBS) <= 7


def test_step_timing_is_diagnostic_only():
    """MBK_STEP_TIMING only adds event records around a step (engine.cpp): the step's
    kernels and copies are the same with and without it."""
    src = (ROOT / "microbeast_amd" / "csrc" / "runtime" / "engine.cpp").read_text()
    assert src.count("MBK_STEP_TIMING") == 1
    # every launch-side use of the timing flag guards an event record only (the one block
    # reads the finished events into the stats)
    guarded = [ln for ln in src.splitlines() if "if (G.timed) ENG_CHECK(" in ln]
    assert guarded and all("hipEventRecord(G.tev[" in ln for ln in guarded)
    assert sum("if (G.timed) {" in ln for ln in src.splitlines()) == 1


def _py(code: str, env: dict) -> str:
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=e, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_force_pg_gloo_world1():
    out = _py("from microbeast_amd.parallel import dist as D\n"
              "i = D.init_distributed(use_cuda=False)\n"
              "print('RESULT', i.enabled, i.backend, i.world_size)\n"
              "D.destroy(i)\n",
              {"MBK_FORCE_PG": "1", "MBK_DIST_BACKEND": "gloo", "WORLD_SIZE": "1", "RANK": "0"})
    line = [ln for ln in out.splitlines() if ln.startswith("RESULT")]
    assert line and line[0].split()[1:] == ["True", "gloo", "1"]


def test_numa_pin_off_keeps_affinity():
    out = _py("import os\nfrom microbeast_amd.parallel import launch\n"
              "a = sorted(os.sched_getaffinity(0))\n"
              "print(launch.pin_rank(0, 8) == a and sorted(os.sched_getaffinity(0)) == a)\n",
              {"MBK_NUMA_PIN": "0"})
    assert out.strip() == "True"
