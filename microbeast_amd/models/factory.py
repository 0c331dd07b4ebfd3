"""Model construction from flags (``--arch``)."""
from __future__ import annotations

import torch

from .agent import Agent
from .gridnet import GridNetAgent

ARCHS = ("impala_flat", "impala_deep", "gridnet")


DTYPES = ("fp32", "bf16", "fp8")


def make_model(flags, device: torch.device | str = "cpu") -> torch.nn.Module:
    """``--dtype``: bf16 / fp8 models run the hand-written bf16 (fp8 acting) MFMA kernels on a
    GPU. fp32 models run plain fp32 PyTorch ops on any device (the HIP kernels are bf16-only,
    so ``hip_kernels`` is off: no bf16 kernel may run under an fp32 flag). The GPU actor
    engine needs the HIP kernels and refuses fp32 (train.py)."""
    if flags.dtype not in DTYPES:
        raise ValueError(f"unknown --dtype {flags.dtype!r}; choose from {DTYPES}")
    s = flags.env_size
    fp32 = flags.dtype == "fp32"
    dt = torch.float32 if fp32 else torch.bfloat16
    kw = dict(compute_dtype=dt, hip_kernels=not fp32)
    if flags.arch == "impala_flat":
        m = Agent((s, s, 27), channels=flags.channel_list(), hidden=flags.hidden, **kw)
    elif flags.arch == "impala_deep":
        # deeper IMPALA-ResNet trunk for large maps (BASELINE config 4, 24x24): 4 stages
        ch = flags.channel_list()
        if len(ch) < 4:
            ch = tuple(ch) + (ch[-1],) * (4 - len(ch))
        m = Agent((s, s, 27), channels=ch, hidden=flags.hidden, **kw)
    elif flags.arch == "gridnet":
        m = GridNetAgent((s, s, 27), **kw)
    else:
        raise ValueError(f"unknown arch {flags.arch!r}; choose from {ARCHS}")
    return m.to(device)
