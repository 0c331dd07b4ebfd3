"""GPU-derived observation planes + action masks == the simulator's own (bit-exact)."""
import pytest
import torch

from microbeast_amd import _native as N
from microbeast_amd.ops.cell_head import OFFS, unpack_mask

pytestmark = pytest.mark.gpu


def _legal(mask_bits, gen):
    mb = unpack_mask(mask_bits)
    n, S, _ = mb.shape
    a = torch.zeros(n, S, 7, dtype=torch.uint8)
    for k in range(7):
        seg = mb[..., OFFS[k]:OFFS[k + 1]].float() + 1e-6
        a[..., k] = torch.multinomial(seg.view(-1, seg.shape[-1]), 1, generator=gen).view(n, S)
    return a


@pytest.mark.parametrize("s", [8, 10, 16, 24])
def test_gpu_mask_matches_simulator(cuda, s):
    rt = N.runtime()
    n, S = 32, s * s
    env = rt.VecEnv(s, n, 400, 3, [0, 1, 2, 3, 5])
    obs = torch.zeros(n, S, dtype=torch.int32)
    mask = torch.zeros(n, S, 3, dtype=torch.int32)
    env.reset(obs.data_ptr(), mask.data_ptr())
    codes = torch.zeros(n, S, dtype=torch.int16)
    res = torch.zeros(n, dtype=torch.int32)
    rew = torch.zeros(n)
    done = torch.zeros(n, dtype=torch.uint8)
    gen = torch.Generator().manual_seed(0)
    k = N.kernels()
    checked = 0
    for step in range(200):
        env.obs_codes(codes.data_ptr(), res.data_ptr())
        cg, rg = codes.to(cuda), res.to(cuda)
        og = torch.empty(n, S, dtype=torch.int32, device=cuda)
        mg = torch.empty(n, S, 3, dtype=torch.int32, device=cuda)
        N.check(k.mbk_decode_obs_mask(cg.data_ptr(), rg.data_ptr(), n, s, s, og.data_ptr(),
                                      mg.data_ptr(), N.stream_ptr()), "decode")
        torch.cuda.synchronize()
        assert torch.equal(og.cpu(), obs), f"obs planes differ at step {step}"
        assert torch.equal(mg.cpu(), mask), f"mask differs at step {step}"
        checked += int((mask != 0).any(-1).sum())
        a = _legal(mask, gen)
        # packed env actions round-trip through the GPU packer and drive the same sim
        a16 = torch.empty(n, S, dtype=torch.int16, device=cuda)
        ag = a.to(cuda)
        N.check(k.mbk_pack_env_actions(ag.data_ptr(), n * S, a16.data_ptr(), N.stream_ptr()), "pack")
        torch.cuda.synchronize()
        env.step(a.data_ptr(), obs.data_ptr(), mask.data_ptr(), rew.data_ptr(), done.data_ptr())
    assert checked > 500


def test_gpu_mask_of_player1_view_matches_simulator(cuda):
    """Self-play: the opponent's mask decoded from its mirrored codes == the sim's p1 mask."""
    rt = N.runtime()
    s, n, S = 10, 16, 100
    env = rt.VecEnv(s, n, 400, 4, [0])
    env.set_external_opponent(True)
    obs = torch.zeros(n, S, dtype=torch.int32)
    mask = torch.zeros(n, S, 3, dtype=torch.int32)
    env.reset(obs.data_ptr(), mask.data_ptr())
    o1 = torch.zeros(n, S, dtype=torch.int32)
    m1 = torch.zeros(n, S, 3, dtype=torch.int32)
    c1 = torch.zeros(n, S, dtype=torch.int16)
    r1 = torch.zeros(n, dtype=torch.int32)
    rew, done = torch.zeros(n), torch.zeros(n, dtype=torch.uint8)
    gen = torch.Generator().manual_seed(2)
    k = N.kernels()
    checked = 0
    for step in range(150):
        env.obs_p1(o1.data_ptr())
        env.mask_p1(m1.data_ptr())
        env.obs_codes_p1(c1.data_ptr(), r1.data_ptr())
        cg, rg = c1.to(cuda), r1.to(cuda)
        og = torch.empty(n, S, dtype=torch.int32, device=cuda)
        mg = torch.empty(n, S, 3, dtype=torch.int32, device=cuda)
        N.check(k.mbk_decode_obs_mask(cg.data_ptr(), rg.data_ptr(), n, s, s, og.data_ptr(),
                                      mg.data_ptr(), N.stream_ptr()), "decode")
        torch.cuda.synchronize()
        assert torch.equal(og.cpu(), o1), f"p1 planes differ at step {step}"
        assert torch.equal(mg.cpu(), m1), f"p1 mask differs at step {step}"
        checked += int((m1 != 0).any(-1).sum())
        a0, a1 = _legal(mask, gen), _legal(m1, gen)
        env.set_opponent_actions(a1.data_ptr())
        env.step(a0.data_ptr(), obs.data_ptr(), mask.data_ptr(), rew.data_ptr(), done.data_ptr())
    assert checked > 200
