"""Fused acting step: a policy step of the flat IMPALA agent in two kernel launches.

The reference acts with ``Agent.get_action`` (model.py:165-216): encoder, then 7*h*w
``CategoricalMasked`` objects sampled one by one in Python. The engine's captured policy graph
replaced that with 6 HIP launches + a scatter copy (decode, stage-0 conv, trunk, network.5 +
critic, head, finale); under a running learner each dependent launch waits for free CU slots,
so the step's latency is set by its launch count (profiles/25). ``mbk_act_step`` does the same
step in TWO launches (``mbk_api.h``):

* A (trunk.hip ``act_trunk_kernel``): codes -> obs bit planes + masks written straight into the
  rollout row, active-pair buckets, stage-0 conv + pool in registers, 14 trunk convs in LDS,
  network.5 + critic (value written into the rollout row);
* B (head.hip ``head_act_kernel``): sparse head sampling, per-env completion counters whose last
  decrement sums the env's log-prob and writes its packed actions; the last workgroup resets the
  buckets and advances the Philox step.

Bit-identical to the graph path (``tests/test_gpu_act.py``). ``ActWorkspace`` holds one policy
lane's pointer block (``MbkActModel``); the GPU engine calls the same C entry per step with the
step's rollout-row pointers (``engine.cpp enqueue_gpu``).
"""
from __future__ import annotations

import ctypes

import torch

from .. import _native as N
from .encoder import encoder_params

c_void_p, c_int = ctypes.c_void_p, ctypes.c_int


class MbkActModel(ctypes.Structure):
    _fields_ = [("w0", c_void_p), ("b0", c_void_p), ("w", c_void_p * 14), ("b", c_void_p * 14),
                ("w5", c_void_p), ("b5", c_void_p), ("wc", c_void_p), ("bc", c_void_p),
                ("Wp", c_void_p), ("bp", c_void_p), ("rng", c_void_p), ("feat", c_void_p),
                ("bucket_cnt", c_void_p), ("bucket", c_void_p), ("cellx", c_void_p),
                ("pending", c_void_p), ("E", c_int), ("H", c_int), ("W", c_int)]


class MbkActStep(ctypes.Structure):
    _fields_ = [("codes", c_void_p), ("res", c_void_p), ("code_list", c_void_p),
                ("obs", c_void_p), ("mask", c_void_p), ("obs2", c_void_p), ("mask2", c_void_p),
                ("action", c_void_p), ("logp", c_void_p), ("value", c_void_p),
                ("act16", c_void_p), ("act_list", c_void_p), ("list_stride", c_int),
                ("reward_src", c_void_p), ("done_src", c_void_p), ("reward_dst", c_void_p),
                ("done_dst", c_void_p), ("step", ctypes.c_uint64), ("abits", c_void_p),
                ("abits2", c_void_p)]


def code_lists(codes: torch.Tensor, res: torch.Tensor, stride: int) -> torch.Tensor:
    """Dense 16-bit codes [E, S] + resources [E] -> the sparse input rows of the fused step
    (word 0 = n | res << 16, then cell | code << 16 per occupied cell in cell order; the
    engine's env workers write this form directly, VecEnv::step_range_lists)."""
    E, S = codes.shape
    c = codes.cpu().to(torch.int64) & 0xFFFF
    nz = c != 0
    cnt = nz.sum(1)
    order = torch.argsort((~nz).to(torch.int8), dim=1, stable=True)  # occupied cells first
    cells = torch.arange(S).expand(E, S)
    ent = torch.gather(cells, 1, order) | (torch.gather(c, 1, order) << 16)
    keep = torch.arange(S)[None, :] < cnt[:, None]
    out = torch.zeros(E, stride, dtype=torch.int64)
    out[:, 0] = cnt | (res.cpu().to(torch.int64) << 16)
    out[:, 1:1 + S] = torch.where(keep, ent, 0)
    out = torch.where(out >= 2 ** 31, out - 2 ** 32, out)  # the uint32 words as int32
    return out.to(torch.int32)


def dense_actions(act_list: torch.Tensor, S: int) -> torch.Tensor:
    """Sparse action rows (word 0 = n, then cell | code << 16) -> dense int16 [E, S] codes."""
    a = act_list.cpu().to(torch.int64) & 0xFFFFFFFF
    E = a.shape[0]
    n = a[:, :1]
    listed = torch.arange(a.shape[1] - 1)[None, :] < n
    ent = a[:, 1:]
    cell = torch.where(listed, ent & 0xFFFF, S)  # unlisted entries land in a dropped column
    out = torch.zeros(E, S + 1, dtype=torch.int64)
    out.scatter_(1, cell, torch.where(listed, ent >> 16, 0))
    return out[:, :S].to(torch.int16)


def supported(model, size: int, fp8: bool = False) -> bool:
    """The fused step covers the headline agent: 16x16 map, (16, 32, 32) trunk, 256 hidden,
    bf16 trunk (the fp8 acting trunk and other shapes keep the captured graph path)."""
    fc = model.network[len(model.channels) + 2] if hasattr(model, "channels") else None
    return (size == 16 and getattr(model, "h", 0) == 16 and getattr(model, "w", 0) == 16
            and tuple(getattr(model, "channels", ())) == (16, 32, 32) and fc is not None
            and fc.out_features == 256 and not fp8 and hasattr(model, "_head"))


class ActWorkspace:
    """Pointer block + workspace of one policy lane for ``mbk_act_step``.

    ``model`` is the lane's inference copy after ``pack_inference`` (its packed buffers and
    parameters keep their addresses: publishes copy into them in place)."""

    def __init__(self, model, E: int, rng: torch.Tensor, device: torch.device):
        assert model._prepacked and model._hip_enc is not None, "pack_inference first"
        enc = model._hip_enc
        assert not enc.fp8 and enc.fused_tail
        S = model.h * model.w
        self.E, self.S = E, S
        head = model._head(device)
        head.ensure_buckets(E)
        self.head = head
        self.feat = torch.empty(E, 256, dtype=torch.bfloat16, device=device)
        self.cellx = torch.zeros(E * S, dtype=torch.int64, device=device)
        self.pending = torch.zeros(2 * E, dtype=torch.int32, device=device)  # + active totals
        # per-cell bucket counters, double-buffered by step parity (mbk_api.h bucket_cnt)
        self.bucket_cnt = torch.zeros(2 * S, dtype=torch.int32, device=device)
        self.rng = rng
        params = encoder_params(model.network, len(model.channels))
        base = enc.packed_fwd.data_ptr()
        ws = [base + 2 * L.w_off for L in enc.layers]
        bs = [p.data_ptr() for p in params[1::2]]
        fc = model.network[len(model.channels) + 2]
        m = MbkActModel()
        m.w0, m.b0 = ws[0], bs[0]
        for i in range(14):
            m.w[i] = ws[i + 1]
            m.b[i] = bs[i + 1]
        m.w5 = model._fc_cache["w5"].data_ptr()
        m.b5 = fc.bias.data_ptr()
        m.wc = model.critic.weight.data_ptr()
        m.bc = model.critic.bias.data_ptr()
        m.Wp, m.bp = head.Wp.data_ptr(), head.bp.data_ptr()
        m.rng = rng.data_ptr()
        m.feat = self.feat.data_ptr()
        m.bucket_cnt, m.bucket = self.bucket_cnt.data_ptr(), head.bucket.data_ptr()
        m.cellx, m.pending = self.cellx.data_ptr(), self.pending.data_ptr()
        m.E, m.H, m.W = E, model.h, model.w
        self.struct = m
        self._keep = (model, params)  # the pointers above stay valid while this lives

    def block(self) -> bytes:
        """The raw MbkActModel bytes (the engine's ``set_act_models``)."""
        return bytes(self.struct)

    def step(self, codes, res, obs, mask, action, logp, value, act16, obs2=None, mask2=None,
             reward=None, done=None, reward_dst=None, done_dst=None, code_list=None,
             act_list=None, step: int | None = None, abits=None, abits2=None) -> None:
        """One fused policy step on the current stream. codes int16 [E, S], res int32 [E]
        (or code_list int32 [E, stride] sparse rows, ``code_lists``); outputs obs int32 [E, S],
        mask int32 [E, S, 3], action uint8 [E, S, 7], logp / value fp32 [E], act16 int16
        [E, S] (or act_list int32 [E, stride] sparse rows); optional second obs / mask
        destination and the reward / done copy of the previous env step. step: the Philox
        step (default: the device counter rng[1], one host sync; the engine counts steps per
        lane itself). abits / abits2: int32 [E, S/32] active-cell bitmap rows to write (the learner's head
        compaction input), abits2 with obs2."""
        s = MbkActStep()
        s.codes, s.res = N.ptr(codes), N.ptr(res)
        s.code_list, s.act_list = N.ptr(code_list), N.ptr(act_list)
        stride = (code_list if code_list is not None else act_list)
        s.list_stride = int(stride.shape[1]) if stride is not None else 0
        s.obs, s.mask = obs.data_ptr(), mask.data_ptr()
        s.obs2, s.mask2 = N.ptr(obs2), N.ptr(mask2)
        s.action, s.logp, s.value = action.data_ptr(), logp.data_ptr(), value.data_ptr()
        s.act16 = N.ptr(act16)
        s.reward_src, s.done_src = N.ptr(reward), N.ptr(done)
        s.step = int(self.rng[1]) if step is None else int(step)
        s.reward_dst, s.done_dst = N.ptr(reward_dst), N.ptr(done_dst)
        s.abits, s.abits2 = N.ptr(abits), N.ptr(abits2)
        N.check(N.kernels().mbk_act_step(ctypes.addressof(self.struct), ctypes.addressof(s),
                                         N.stream_ptr()), "act_step")
