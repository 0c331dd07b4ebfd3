"""Host-code sanitizer runs of the native runtime (tools/sanitize.sh): MPMC index ring,
seqlock weight slot and multi-threaded self-play env stepping under ASan+UBSan and TSan.
GPU sanitizers / XNACK are unavailable on this pool, so only host code is instrumented."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("mode", ["asan", "tsan"])
def test_host_runtime_under_sanitizer(mode, tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize.sh"), mode], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "host stress: all ok" in r.stdout
