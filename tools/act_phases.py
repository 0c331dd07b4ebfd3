#!/usr/bin/env python
"""Where the fused acting step's time goes (ops/act.py, mbk_act_step) on one MI355X.

Runs the two launches standalone on E envs of real simulator codes (sparse rows in pinned host
memory, as the engine feeds them, or in device memory), times each launch with HIP events, then
re-runs launch A with the diagnostic phase stamps (trunk.hip ACT_STAMP) and prints the mean
share of each prologue / trunk phase over the workgroups' first tiles.

  python tools/act_phases.py [--envs 8192] [--steps 20] [--device_rows]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# stamp intervals of wave 0's first tile (act_trunk_w_kernel): its own 2 envs through the
# trunk, then the tile-wide end (bucket reservation, FC + critic, bucket entries)
PHASES_WAVE = (["rows + codes", "decode", "conv0 + pool + halos"]
               + [("pool + halos + " if l in (5, 10) else "") + f"conv {l}" for l in range(14)]
               + ["(trunk end)", "barrier 1 wait", "FC + critic + bucket entries"])


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=8192)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warm", type=int, default=30, help="env steps before sampling codes")
    p.add_argument("--device_rows", action="store_true", help="sparse rows in HBM, not pinned")
    p.add_argument("--spread", action="store_true",
                   help="roll every env's map by its own random (dy, dx): the active cells then "
                        "spread over the whole map as in a settled run (~100 pairs per cell) "
                        "instead of sitting on the same few cells of every env")
    p.add_argument("--lib", default=None, help="variant library dir (tools/variant.py)")
    p.add_argument("--settled_rows", action="store_true",
                   help="pad every row with (empty cell, code 0) entries -- a no-op for the "
                        "decode -- to the settled bench's occupancy (mean ~21 cells per env, "
                        "p90 30, ~7 %% over 31: bench.py occupied_cells_per_env), so launch A's "
                        "row reads cost what they cost in the bench")
    a = p.parse_args()
    from tools.variant import use_lib
    use_lib(a.lib)
    from microbeast_amd import _native as N
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.act import ActWorkspace, MbkActStep

    dev = torch.device("cuda", 0)
    rt = N.runtime()
    E, S = a.envs, 256
    env = rt.VecEnv(16, E, 2000, 1, [0, 0, 0, 1, 2, 3])
    obs = torch.zeros(E, S, dtype=torch.int32)
    mask = torch.zeros(E, S, 3, dtype=torch.int32)
    env.reset(obs.data_ptr(), mask.data_ptr())
    zero = torch.zeros(E, S, 7, dtype=torch.uint8)
    rew, done = torch.zeros(E), torch.zeros(E, dtype=torch.uint8)
    for _ in range(a.warm):  # no-op agent: the bots play, units spread over the map
        env.step(zero.data_ptr(), obs.data_ptr(), mask.data_ptr(), rew.data_ptr(), done.data_ptr())
    stride = S + 4
    rows = torch.zeros(E, stride, dtype=torch.int32)
    codes = torch.zeros(E, S, dtype=torch.int16)
    res = torch.zeros(E, dtype=torch.int32)
    env.obs_codes(codes.data_ptr(), res.data_ptr())
    if a.spread:
        g = torch.Generator().manual_seed(5)
        sh = torch.randint(0, 16, (E, 2), generator=g)
        yy = (torch.arange(16)[None, :, None] - sh[:, 0, None, None]) % 16
        xx = (torch.arange(16)[None, None, :] - sh[:, 1, None, None]) % 16
        codes = torch.gather(codes.view(E, S), 1, (yy * 16 + xx).view(E, S))
    c = codes.to(torch.int64) & 0xFFFF
    nz = c != 0
    cnt = nz.sum(1)
    rows[:, 0] = (cnt | (res.to(torch.int64) << 16)).to(torch.int32)
    cells = torch.arange(S).expand(E, S)
    order = torch.argsort((~nz).to(torch.int8), dim=1, stable=True)  # occupied cells first
    ent = (torch.gather(cells, 1, order) | (torch.gather(c, 1, order) << 16))
    keep = torch.arange(S)[None, :] < cnt[:, None]
    rows[:, 1:1 + S] = torch.where(keep, ent, 0).to(torch.int32)
    if a.settled_rows:
        g = torch.Generator().manual_seed(9)
        want = (torch.randn(E, generator=g) * 7.0 + 20.5).clamp(11, 40).round().to(torch.int64)
        for e in range(E):
            n = int(cnt[e])
            k = max(0, int(want[e]) - n)
            empty = torch.nonzero(c[e] == 0).view(-1)[:k]
            rows[e, 1 + n:1 + n + len(empty)] = empty.to(torch.int32)
            rows[e, 0] = (int(rows[e, 0]) & ~0xFFFF) | (n + len(empty))
        occ = rows[:, 0] & 0xFFFF
        print(f"settled rows: occupied mean {occ.float().mean():.1f}, "
              f"over 31: {float((occ > 31).float().mean()):.3f}")
    rows = rows.to(dev) if a.device_rows else rows.pin_memory()
    print(f"occupied cells per env: mean {cnt.float().mean():.1f} max {int(cnt.max())}; "
          f"active (idle own units) {float((mask != 0).any(-1).float().sum(1).mean()):.2f}")

    torch.manual_seed(0)
    m = Agent((16, 16, 27))
    torch.nn.init.normal_(m.actor.weight, std=0.05)
    m = m.to(dev).eval()
    m.pack_inference(dev)
    rng = torch.tensor([1, 0], dtype=torch.int64, device=dev)
    ws = ActWorkspace(m, E, rng, dev)
    o = torch.empty(E, S, dtype=torch.int32, device=dev)
    mk = torch.empty(E, S, 3, dtype=torch.int32, device=dev)
    act = torch.empty(E, S, 7, dtype=torch.uint8, device=dev)
    lp = torch.empty(E, device=dev)
    v = torch.empty(E, device=dev)
    al = torch.zeros(E, stride, dtype=torch.int32).pin_memory()
    st = MbkActStep()
    st.code_list, st.act_list, st.list_stride = rows.data_ptr(), al.data_ptr(), stride
    st.obs, st.mask, st.action, st.logp, st.value = (o.data_ptr(), mk.data_ptr(), act.data_ptr(),
                                                     lp.data_ptr(), v.data_ptr())
    k = N.kernels()
    args = (ctypes.addressof(ws.struct), ctypes.addressof(st))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ta = tb = 0.0
    for i in range(a.steps + 3):
        st.step = i  # the Philox step selects the bucket counters' half (step parity)
        ev[0].record()
        N.check(k.mbk_act_trunk(*args, N.stream_ptr()), "act_trunk")
        ev[1].record()
        N.check(k.mbk_act_head(*args, N.stream_ptr()), "act_head")
        ev[2].record()
        torch.cuda.synchronize()
        if i >= 3:
            ta += ev[0].elapsed_time(ev[1])
            tb += ev[1].elapsed_time(ev[2])
    n = a.steps
    print(f"launch A (decode + trunk + critic) {1e3 * ta / n:.1f} us, launch B (head + finale) "
          f"{1e3 * tb / n:.1f} us, rows in "
          f"{'HBM' if a.device_rows else 'pinned host memory'}")
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    stamps = torch.zeros(ncu * 4 * 32 * 64, dtype=torch.int64, device=dev)
    nst = k.mbk_act_set_stamps(stamps.data_ptr())
    st.step = a.steps + 3
    N.check(k.mbk_act_trunk(*args, N.stream_ptr()), "act_trunk (stamped)")
    torch.cuda.synchronize()
    k.mbk_act_set_stamps(None)
    names = PHASES_WAVE
    nb = stamps.numel() // (nst * 64)
    t = stamps[:nb * nst * 64].view(nb, nst, 64)[:, :, 0].cpu().double()
    t = t[t[:, 0] > 0][:, :len(names) + 1]
    d = (t[:, 1:] - t[:, :-1]) * 10.0 / 1e3  # 100 MHz ticks -> us
    tot = float(d.sum(1).mean())
    print(f"first tile of {len(t)} workgroups: {tot:.1f} us")
    for i, name in enumerate(names):
        print(f"  {name:18s} {float(d[:, i].mean()):7.2f} us  {float(d[:, i].mean()) / tot:6.1%}")


if __name__ == "__main__":
    main()
