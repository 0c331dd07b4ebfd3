"""Self-play env path: packed two-player fast path == validated reference path."""
import numpy as np
import torch

from microbeast_amd import _native as N
from microbeast_amd.ops.cell_head import OFFS, unpack_mask


def _legal(mask_bits, gen):
    mb = unpack_mask(mask_bits)
    n, S, _ = mb.shape
    a = torch.zeros(n, S, 7, dtype=torch.uint8)
    for k in range(7):
        seg = mb[..., OFFS[k]:OFFS[k + 1]].float() + 1e-6
        a[..., k] = torch.multinomial(seg.view(-1, seg.shape[-1]), 1, generator=gen).view(n, S)
    return a


def pack_actions(a: torch.Tensor) -> torch.Tensor:
    """numpy mirror of mbr::pack_env_action (include/microrts_rules.h)."""
    a = a.numpy().astype(np.int32)
    t = np.where(a[..., 0] < 6, a[..., 0], 0)
    dirs = np.zeros_like(t)
    for k in range(1, 5):
        dirs = np.where(t == k, a[..., k], dirs)
    v = t | ((dirs & 3) << 3) | ((a[..., 5] & 7) << 5) | ((a[..., 6] & 63) << 8)
    return torch.from_numpy(v.astype(np.int16))


def test_selfplay_fast_path_matches_validated_path():
    rt = N.runtime()
    s, n, S = 10, 6, 100
    A = rt.VecEnv(s, n, 300, 5, [0])
    B = rt.VecEnv(s, n, 300, 5, [0])
    A.set_external_opponent(True)
    B.set_external_opponent_range(0, n, True)
    B.set_validate(False)
    obs = torch.zeros(n, S, dtype=torch.int32)
    mask = torch.zeros(n, S, 3, dtype=torch.int32)
    mask1 = torch.zeros(n, S, 3, dtype=torch.int32)
    A.reset(obs.data_ptr(), mask.data_ptr())
    B.reset(0, 0)
    rA, dA = torch.zeros(n), torch.zeros(n, dtype=torch.uint8)
    rB, dB = torch.zeros(n), torch.zeros(n, dtype=torch.uint8)
    cA, resA = torch.zeros(n, S, dtype=torch.int16), torch.zeros(n, dtype=torch.int32)
    cA1, resA1 = torch.zeros(n, S, dtype=torch.int16), torch.zeros(n, dtype=torch.int32)
    cB, resB = torch.zeros(n, S, dtype=torch.int16), torch.zeros(n, dtype=torch.int32)
    cB1, resB1 = torch.zeros(n, S, dtype=torch.int16), torch.zeros(n, dtype=torch.int32)
    gen = torch.Generator().manual_seed(1)
    dones = 0
    for step in range(700):
        A.mask_p1(mask1.data_ptr())
        a0, a1 = _legal(mask, gen), _legal(mask1, gen)
        A.set_opponent_actions(a1.data_ptr())
        A.step(a0.data_ptr(), obs.data_ptr(), mask.data_ptr(), rA.data_ptr(), dA.data_ptr())
        p0, p1 = pack_actions(a0), pack_actions(a1)
        B.step_codes_sp(p0.data_ptr(), p1.data_ptr(), cB.data_ptr(), resB.data_ptr(),
                        cB1.data_ptr(), resB1.data_ptr(), rB.data_ptr(), dB.data_ptr(), 7)
        A.obs_codes(cA.data_ptr(), resA.data_ptr())
        A.obs_codes_p1(cA1.data_ptr(), resA1.data_ptr())
        assert torch.equal(cA, cB) and torch.equal(resA, resB), step
        assert torch.equal(cA1, cB1) and torch.equal(resA1, resB1), step
        assert torch.equal(rA, rB) and torch.equal(dA, dB), step
        dones += int(dA.sum())
    assert dones > 0
    eb, ea = B.drain_episodes(), A.drain_episodes()
    assert len(ea) == len(eb) == dones
    assert all(e[4] == 7 for e in eb)
    assert [e[:4] for e in ea] == [e[:4] for e in eb]


def test_player1_codes_are_the_mirrored_view():
    rt = N.runtime()
    s, n, S = 8, 2, 64
    env = rt.VecEnv(s, n, 300, 9, [0])
    env.set_external_opponent(True)
    env.reset(0, 0)
    c0, r0 = torch.zeros(n, S, dtype=torch.int16), torch.zeros(n, dtype=torch.int32)
    c1, r1 = torch.zeros(n, S, dtype=torch.int16), torch.zeros(n, dtype=torch.int32)
    env.obs_codes(c0.data_ptr(), r0.data_ptr())
    env.obs_codes_p1(c1.data_ptr(), r1.data_ptr())
    owner = lambda c: (c.int() >> 6) & 3  # noqa: E731
    # the symmetric start map: the rotated p1 view equals p0's view
    rot = c1.view(n, s, s).flip(1).flip(2).reshape(n, S)
    swapped = torch.where(owner(rot) == 1, 2, torch.where(owner(rot) == 2, 1, owner(rot)))
    assert torch.equal(swapped, owner(c0))
    assert torch.equal(c1, c0)  # symmetric start: identical from both seats


def _rows_to_dense(rows: torch.Tensor, S: int) -> torch.Tensor:
    """sparse rows (word 0 = n | res << 16, then cell | code << 16) -> dense int16 codes"""
    from microbeast_amd.ops.act import dense_actions
    r = rows.clone()
    r[:, 0] &= 0xFFFF
    return dense_actions(r, S)


def _dense_to_rows(codes: torch.Tensor, stride: int) -> torch.Tensor:
    from microbeast_amd.ops.act import code_lists
    return code_lists(codes, torch.zeros(codes.shape[0], dtype=torch.int32), stride)


def test_selfplay_sparse_rows_match_dense_step():
    """The engine's fused self-play form (VecEnv::step_range_lists_sp: both players' sparse
    action rows in, both players' code rows out) == the dense packed self-play step."""
    rt = N.runtime()
    s, n, S = 10, 6, 100
    stride = S + 4
    B = rt.VecEnv(s, n, 300, 5, [0])
    C = rt.VecEnv(s, n, 300, 5, [0])
    for e in (B, C):
        e.set_external_opponent_range(0, n, True)
        e.set_validate(False)
        e.reset(0, 0)
    A = rt.VecEnv(s, n, 300, 5, [0])  # masks for legal random actions (validated twin)
    A.set_external_opponent(True)
    obs = torch.zeros(n, S, dtype=torch.int32)
    mask = torch.zeros(n, S, 3, dtype=torch.int32)
    mask1 = torch.zeros(n, S, 3, dtype=torch.int32)
    A.reset(obs.data_ptr(), mask.data_ptr())
    rA, dA = torch.zeros(n), torch.zeros(n, dtype=torch.uint8)
    rB, dB = torch.zeros(n), torch.zeros(n, dtype=torch.uint8)
    rC, dC = torch.zeros(n), torch.zeros(n, dtype=torch.uint8)
    cB, resB = torch.zeros(n, S, dtype=torch.int16), torch.zeros(n, dtype=torch.int32)
    cB1, resB1 = torch.zeros(n, S, dtype=torch.int16), torch.zeros(n, dtype=torch.int32)
    lC = torch.zeros(n, stride, dtype=torch.int32)
    lC1 = torch.zeros(n, stride, dtype=torch.int32)
    C.code_lists(lC.data_ptr(), stride, 0)
    C.code_lists(lC1.data_ptr(), stride, 1)
    B.obs_codes(cB.data_ptr(), resB.data_ptr())
    B.obs_codes_p1(cB1.data_ptr(), resB1.data_ptr())
    assert torch.equal(_rows_to_dense(lC, S), cB) and torch.equal(_rows_to_dense(lC1, S), cB1)
    gen = torch.Generator().manual_seed(3)
    dones = 0
    for step in range(600):
        A.mask_p1(mask1.data_ptr())
        a0, a1 = _legal(mask, gen), _legal(mask1, gen)
        A.set_opponent_actions(a1.data_ptr())
        A.step(a0.data_ptr(), obs.data_ptr(), mask.data_ptr(), rA.data_ptr(), dA.data_ptr())
        p0, p1 = pack_actions(a0), pack_actions(a1)
        B.step_codes_sp(p0.data_ptr(), p1.data_ptr(), cB.data_ptr(), resB.data_ptr(),
                        cB1.data_ptr(), resB1.data_ptr(), rB.data_ptr(), dB.data_ptr(), 7)
        ap0, ap1 = _dense_to_rows(p0, stride), _dense_to_rows(p1, stride)
        C.step_lists_sp(ap0.data_ptr(), ap1.data_ptr(), lC.data_ptr(), lC1.data_ptr(), stride,
                        rC.data_ptr(), dC.data_ptr(), 7)
        assert torch.equal(_rows_to_dense(lC, S), cB), step
        assert torch.equal(_rows_to_dense(lC1, S), cB1), step
        assert torch.equal(lC[:, 0] >> 16, resB) and torch.equal(lC1[:, 0] >> 16, resB1), step
        assert torch.equal(rB, rC) and torch.equal(dB, dC), step
        dones += int(dB.sum())
    assert dones > 0
    eb, ec = B.drain_episodes(), C.drain_episodes()
    assert [e[:5] for e in eb] == [e[:5] for e in ec] and all(e[4] == 7 for e in ec)
