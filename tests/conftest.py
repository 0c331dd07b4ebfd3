import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: multi-process / long CPU tests")
    # the pixel-major GridNet ops' CPU emulation is test code (tests/pixconv_emulation.py)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import pixconv_emulation
    from microbeast_amd.ops import pixconv
    pixconv.set_emulation(pixconv_emulation)


WGRAD_QUEUE_SITE = 4  # common.h kQueueWgrad


@pytest.fixture(scope="session")
def rt():
    from microbeast_amd import _native as N
    return N.runtime()


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from microbeast_amd import _native as N
    N.kernels()  # fail loudly if the HIP library is missing
    # the suite pins kernels and whole updates bit for bit across separate runs; the weight
    # gradient's work queue (conv.hip, on in training and the bench) sums each workgroup's
    # rounds in a run-dependent order, so the suite runs it with the static stride except
    # where a test turns it on (test_gpu_conv.py::test_wgrad_queue_matches_static)
    N.check(N.kernels().mbk_set_work_queue_site(WGRAD_QUEUE_SITE, 0), "queue site")
    return torch.device("cuda", 0)
