"""Model construction from flags (``--arch``)."""
from __future__ import annotations

import torch

from .agent import Agent
from .gridnet import GridNetAgent

ARCHS = ("impala_flat", "impala_deep", "gridnet")


def make_model(flags, device: torch.device | str = "cpu") -> torch.nn.Module:
    s = flags.env_size
    dt = torch.bfloat16 if flags.dtype in ("bf16", "fp8") else torch.float32
    if flags.arch == "impala_flat":
        m = Agent((s, s, 27), channels=flags.channel_list(), hidden=flags.hidden, compute_dtype=dt)
    elif flags.arch == "impala_deep":
        # deeper IMPALA-ResNet trunk for large maps (BASELINE config 4, 24x24): 4 stages
        ch = flags.channel_list()
        if len(ch) < 4:
            ch = tuple(ch) + (ch[-1],) * (4 - len(ch))
        m = Agent((s, s, 27), channels=ch, hidden=flags.hidden, compute_dtype=dt)
    elif flags.arch == "gridnet":
        m = GridNetAgent((s, s, 27), compute_dtype=dt)
    else:
        raise ValueError(f"unknown arch {flags.arch!r}; choose from {ARCHS}")
    return m.to(device)
