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


def row_gather(src: torch.Tensor, idx: torch.Tensor, k: int, out: torch.Tensor | None = None):
    """out[i] = src[idx[i]] for i < k (rows along dim 0; idx: device int64)."""
    row = src[0].numel() * src.element_size()
    if out is None:
        out = torch.empty((k,) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    assert src.is_contiguous() and out.is_contiguous() and idx.dtype == torch.int64
    N.check(N.kernels().mbk_row_gather(src.data_ptr(), out.data_ptr(), idx.data_ptr(), k, row,
                                       N.stream_ptr()), "row_gather")
    return out


def zero_(t: torch.Tensor) -> torch.Tensor:
    """t.zero_() for a contiguous tensor (hipMemsetAsync on the GPU, no ATen fill kernel)."""
    if not t.is_cuda:
        return t.zero_()
    assert t.is_contiguous()
    N.check(N.kernels().mbk_memset(t.data_ptr(), 0, t.numel() * t.element_size(),
                                   N.stream_ptr()), "memset")
    return t


def zeros(*shape, dtype=torch.float32, device=None) -> torch.Tensor:
    """torch.zeros without an ATen fill kernel on the GPU (hipMemsetAsync)."""
    if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
        shape = tuple(shape[0])
    return zero_(torch.empty(shape, dtype=dtype, device=device))


def full(shape, value: float, dtype=torch.float32, device=None) -> torch.Tensor:
    """constant tensor built on the host and DMA'd (no ATen fill kernel on the GPU)"""
    t = torch.full(shape, value, dtype=dtype)
    return t.to(device) if device is not None else t
