"""Batched device copies through one kernel launch (``copy.hip``)."""
from __future__ import annotations

import ctypes

import torch

from .. import _native as N

MAX_SEGS = 16


class _Seg(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("bytes", ctypes.c_uint64)]


def multi_copy(pairs: list[tuple[torch.Tensor, torch.Tensor]]) -> None:
    """dst.copy_(src) for every (src, dst) pair, contiguous same-size tensors, one launch per 16."""
    k = N.kernels()
    st = N.stream_ptr()
    for i in range(0, len(pairs), MAX_SEGS):
        chunk = pairs[i:i + MAX_SEGS]
        arr = (_Seg * len(chunk))()
        for j, (s, d) in enumerate(chunk):
            nb = s.numel() * s.element_size()
            assert s.is_contiguous() and d.is_contiguous() and nb == d.numel() * d.element_size()
            arr[j] = _Seg(s.data_ptr(), d.data_ptr(), nb)
        N.check(k.mbk_multi_copy(ctypes.cast(arr, ctypes.c_void_p), len(chunk), st), "multi_copy")
