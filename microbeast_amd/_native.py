"""Loader for the in-tree native libraries (built by ``csrc/build.py``).

* ``kernels()`` — ctypes handle to ``_lib/libmbk_kernels.so`` (HIP, gfx950).
* ``runtime()`` — the pybind11 ``_mbrt`` module (env, rings, GPU engine).

torch is imported first on purpose: the ROCm torch wheel ships its own
``libamdhip64.so.7``; loading ours afterwards makes the dynamic loader reuse
that already-loaded HIP runtime (same SONAME) instead of mapping a second one.

GPU ops fail loudly when the kernel library is missing on a GPU box — there
is no silent PyTorch fallback for device tensors.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import sys
import threading
from pathlib import Path

import torch  # noqa: F401  (must precede the HIP libraries, see module doc)

_LIB = Path(__file__).resolve().parent / "_lib"
_lock = threading.Lock()
_kern = None
_rt = None

c_void_p, c_int, c_int64, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float

_SIGS = {
    "mbk_multi_copy": [c_void_p, c_int, c_void_p],
    "mbk_comm_standin": [c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p],
    "mbk_row_gather": [c_void_p, c_void_p, c_void_p, c_int, c_int64, c_void_p],
    "mbk_memset": [c_void_p, c_int, c_int64, c_void_p],
    "mbk_masked_cell_fwd": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int64,
                            c_void_p, c_void_p, c_void_p],
    "mbk_masked_cell_bwd": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                            c_int64, c_void_p, c_int, c_void_p],
    "mbk_row_sum": [c_void_p, c_int64, c_int, c_void_p, c_void_p],
    "mbk_masked_cell_fwd_pbc": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                c_int, c_int64, c_void_p, c_void_p, c_void_p],
    "mbk_masked_cell_bwd_pbc": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_int64, c_void_p, c_void_p],
    "mbk_pconv": [c_void_p, c_void_p],
    "mbk_imgconv": [c_void_p, c_int, c_void_p],
    "mbk_imgwgrad": [c_void_p, c_int, c_void_p],
    "mbk_imgwgrad_parts": [],
    "mbk_cells_nchunk": [c_int],
    "mbk_cells_compact": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "mbk_rows_colsum": [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p],
    "mbk_masked_cell_rows_fwd": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                                 c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    "mbk_masked_cell_rows_bwd": [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "mbk_pwgrad": [c_void_p, c_void_p],
    "mbk_pwgrad_all": [c_void_p, c_void_p],
    "mbk_pwgrad_all_parts": [c_int, c_int, c_int],
    "mbk_pwgrad_parts": [c_int, c_int, c_int, c_int],
    "mbk_reduce_map": [c_void_p, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p],
    "mbk_reduce_inv": [c_void_p, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                       c_void_p],
    "mbk_ppool_fwd": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "mbk_ppool_bwd": [c_void_p, c_int64, c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                      c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "mbk_rng_advance": [c_void_p, c_void_p],
    "mbk_vtrace": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                   c_float, c_float, c_float, c_float, c_float, c_float, c_float, c_void_p,
                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "mbk_grad_clip_scale": [c_void_p, c_int64, c_float, c_float, c_void_p, c_void_p, c_void_p],
    "mbk_adam": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float,
                 c_float, c_float, c_float, c_int64, c_void_p, c_float, c_void_p],
    "mbk_to_bf16": [c_void_p, c_int64, c_void_p, c_void_p],
    "mbk_from_bf16": [c_void_p, c_int64, c_void_p, c_void_p],
    "mbk_conv_fwd": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                     c_void_p],
    "mbk_conv_fwd_fp8": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "mbk_conv_pack_fp8": [c_void_p, c_int, c_void_p],
    "mbk_pool_bwd_idx": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "mbk_conv_wgrad": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "mbk_conv_wgrad_parts": [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int],
    "mbk_pool_conv_bwd_parts": [c_int, c_int, c_int, c_int, c_int],
    "mbk_pool_conv_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                          c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "mbk_pool_conv_bwd_partial_floats": [c_int, c_int, c_int],
    "mbk_conv_set_grid_cap": [c_int],
    "mbk_set_learner_occupancy": [c_int, c_int],
    "mbk_set_work_queues": [c_int],
    "mbk_set_work_queue_site": [c_int, c_int],
    "mbk_conv0_row_set": [c_int],
    "mbk_fc_wgrad_parts": [c_int, c_int, c_int],
    "mbk_fc_wgrad": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
                     c_void_p],
    "mbk_fc_fwd": [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                   c_void_p, c_void_p, c_void_p],
    "mbk_gemm_nt": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                    c_int, c_int, c_int, c_int, c_void_p],
    "mbk_wgrad_reduce": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                         c_void_p],
    "mbk_wgrad_reduce_batch": [c_void_p, c_int, c_void_p],
    "mbk_pool_bwd": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "mbk_conv_pack": [c_void_p, c_int, c_void_p],
    "mbk_head_compact": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "mbk_head_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                     c_void_p, c_void_p, c_int, c_void_p],
    "mbk_fc_wgrad_wide_parts": [c_int, c_int, c_int],
    "mbk_fc_wgrad_wide": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                          c_void_p, c_void_p, c_void_p],
    "mbk_head_score": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                       c_void_p, c_void_p],
    "mbk_head_pair_rowsum": [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                             c_void_p, c_void_p],
    "mbk_head_bwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                     c_void_p, c_void_p, c_void_p],
    "mbk_head_dx_gather": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p],
    "mbk_head_dx_value_parts": [c_int],
    "mbk_head_dx_value": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                          c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p],
    "mbk_head_pack": [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p],
    "mbk_decode_obs_mask": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "mbk_decode_obs_mask_bucket": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "mbk_head_units": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                       c_void_p],
    "mbk_row_sum_rng": [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p],
    "mbk_row_sum_pack": [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_int, c_void_p],
    "mbk_head_fwd_counts": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    "mbk_trunk_tail": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    "mbk_trunk_tail_fp8": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                           c_void_p],
    "mbk_trunk_tail_fc": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                          c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p],
    "mbk_pack_env_actions": [c_void_p, c_int64, c_void_p, c_void_p],
    "mbk_res_bwd16_parts": [c_int, c_int, c_int, c_int],
    "mbk_res_bwd32_parts": [c_int, c_int, c_int, c_int],
    "mbk_res_bwd32_partial_floats": [c_int],
    "mbk_res_bwd32": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                      c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                      c_int, c_void_p],
    "mbk_res_fwd16": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                      c_int, c_int, c_int, c_void_p],
    "mbk_res_fwd16_stage": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                            c_void_p],
    "mbk_res_blk32_fwd": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                          c_void_p],
    "mbk_pool_conv_fwd4": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    "mbk_res_blk32_fwd_wave": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                               c_int, c_void_p],
    "mbk_res_bwd32_team_parts": [c_int, c_int, c_int],
    "mbk_res_bwd32_team": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_int, c_int, c_int, c_int, c_void_p],
    "mbk_res_bwd16_partial_floats": [c_int],
    "mbk_res_bwd16": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                      c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                      c_int, c_void_p],
    # gridnet.hip
    "mbk_bits_pad": [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "mbk_colsum_parts": [c_int64],
    "mbk_colsum": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p,
                   c_void_p],
    "mbk_map_gather": [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    "mbk_value_bwd_parts": [c_int],
    "mbk_value_bwd": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                      c_int, c_int, c_void_p],
    "mbk_fc_wgrad_ex": [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int,
                        c_int, c_void_p],
    # fused acting step (ops/act.py): (const MbkActModel*, const MbkActStep*, stream)
    "mbk_act_step": [c_void_p, c_void_p, c_void_p],
    "mbk_act_trunk": [c_void_p, c_void_p, c_void_p],
    "mbk_act_head": [c_void_p, c_void_p, c_void_p],
    "mbk_act_set_stamps": [c_void_p],
    "mbk_rows_to_codes": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p],
    "mbk_codes_to_rows": [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p],
    "mbk_gemm_nt_mask": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                         c_int, c_int, c_int, c_void_p, c_void_p],
}
_RESTYPE = {"mbk_res_bwd16_partial_floats": c_int64, "mbk_res_bwd32_partial_floats": c_int64,
            "mbk_pool_conv_bwd_partial_floats": c_int64}


def _ensure_built() -> None:
    kl = _LIB / "libmbk_kernels.so"
    rts = list(_LIB.glob("_mbrt*.so"))
    if kl.exists() and rts and os.environ.get("MBK_REBUILD", "0") != "1":
        return
    from .csrc import build as _b

    _b.build()


def kernels():
    """ctypes handle to libmbk_kernels.so (builds it if missing)."""
    global _kern
    if _kern is not None:
        return _kern
    with _lock:
        if _kern is None:
            _ensure_built()
            lib = ctypes.CDLL(str(_LIB / "libmbk_kernels.so"), mode=ctypes.RTLD_GLOBAL)
            for name, args in _SIGS.items():
                fn = getattr(lib, name)  # a missing symbol is a build error: fail loudly
                fn.argtypes = args
                fn.restype = _RESTYPE.get(name, c_int)
            _kern = _Checked(lib)
    return _kern


class _Checked:
    """Only signature-declared launchers are reachable (ctypes' default int
    conversion would silently truncate 64-bit device pointers)."""

    def __init__(self, lib):
        self._lib = lib

    def __getattr__(self, name):
        if name not in _SIGS:
            raise AttributeError(f"{name}: no ctypes signature declared in _native._SIGS")
        return getattr(self._lib, name)


def runtime():
    """The _mbrt pybind11 module (builds it if missing)."""
    global _rt
    if _rt is not None:
        return _rt
    with _lock:
        if _rt is None:
            _ensure_built()
            kernels_path = _LIB / "libmbk_kernels.so"
            ctypes.CDLL(str(kernels_path), mode=ctypes.RTLD_GLOBAL)
            cands = sorted(_LIB.glob("_mbrt*.so"))
            if not cands:
                raise ImportError("microbeast_amd native runtime (_mbrt) not built")
            spec = importlib.util.spec_from_file_location("microbeast_amd._lib._mbrt", cands[0])
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["microbeast_amd._lib._mbrt"] = mod
            _rt = mod
    return _rt


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


def stream_ptr(stream: torch.cuda.Stream | None = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def loaded_libraries() -> list[str]:
    """In-tree native libraries mapped into this process (for smoke checks)."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if str(_LIB) in line:
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out
