#!/usr/bin/env python
"""How the policy step's GPU cost and the env's CPU cost scale with the share of ACTIVE cells
(cells holding an idle own unit: the sparse head samples exactly those).

The headline bench runs random-init weights, whose uniform policy keeps ~0.5 % of cells active
on 16x16; a trained policy builds more units (the r3b1L CLI run averaged 10.96 M frames/s
against the bench's ~14 M). This tool prices both sides at 0.5 / 2 / 5 % active cells:

* GPU: the policy step (ops/act.py, mbk_act_step, launch A + launch B) on
  E envs of real simulator codes with extra own idle workers dropped on empty cells until each
  env has the target number of active cells (the step's decode recomputes the masks from the
  codes, so the head samples exactly those cells);
* CPU: one VecEnv step per env (the engine's env workers' unit of work), timed on real games
  played by a uniform-random agent (its units accumulate over an episode), binned by the
  active share the step started from.

    python tools/active_sweep.py [--envs 8192] [--cpu_only]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

S = 256
WORKER, OWN = 4, 1  # include/microrts_rules.h: type WORKER, owner 1 = the observing player


def worker_code() -> int:
    """an own idle worker with 1 hp and nothing carried (cell_code(hp, res, owner, type, act))"""
    return 1 | (0 << 3) | (OWN << 6) | (WORKER << 8) | (0 << 11)


def synthetic_rows(E: int, active: int, seed: int):
    """sparse input rows (ops/act.py code_lists form) of E warmed-up 16x16 envs with extra own
    idle workers on empty cells: ~``active`` active cells per env"""
    from microbeast_amd import _native as N
    rt = N.runtime()
    env = rt.VecEnv(16, E, 2000, seed, [0, 0, 0, 1, 2, 3])
    obs = torch.zeros(E, S, dtype=torch.int32)
    mask = torch.zeros(E, S, 3, dtype=torch.int32)
    env.reset(obs.data_ptr(), mask.data_ptr())
    zero = torch.zeros(E, S, 7, dtype=torch.uint8)
    rew, done = torch.zeros(E), torch.zeros(E, dtype=torch.uint8)
    for _ in range(30):
        env.step(zero.data_ptr(), obs.data_ptr(), mask.data_ptr(), rew.data_ptr(), done.data_ptr())
    codes = torch.zeros(E, S, dtype=torch.int16)
    res = torch.zeros(E, dtype=torch.int32)
    env.obs_codes(codes.data_ptr(), res.data_ptr())
    c = codes.numpy().astype(np.int64) & 0xFFFF
    rng = np.random.default_rng(seed)
    base_active = (mask.numpy() != 0).any(-1).sum(1)
    for e in range(E):
        need = max(0, active - int(base_active[e]))
        empty = np.flatnonzero(c[e] == 0)
        if need:
            c[e, rng.choice(empty, size=min(need, len(empty)), replace=False)] = worker_code()
    res[:] = 50  # enough resources for every produce / build option
    from microbeast_amd.ops.act import code_lists
    return code_lists(torch.from_numpy(c.astype(np.int16)), res, S + 4)


def gpu_sweep(E: int, fracs, steps: int) -> list[dict]:
    from microbeast_amd import _native as N
    from microbeast_amd.models.agent import Agent
    from microbeast_amd.ops.act import ActWorkspace, MbkActStep
    dev = torch.device("cuda", 0)
    k = N.kernels()
    torch.manual_seed(0)
    m = Agent((16, 16, 27))
    torch.nn.init.normal_(m.actor.weight, std=0.05)
    m = m.to(dev).eval()
    m.pack_inference(dev)
    rng = torch.tensor([1, 0], dtype=torch.int64, device=dev)
    ws = ActWorkspace(m, E, rng, dev)
    stride = S + 4
    out = []
    for f in fracs:
        rows = synthetic_rows(E, max(1, round(f * S)), seed=11).pin_memory()
        o = torch.empty(E, S, dtype=torch.int32, device=dev)
        mk = torch.empty(E, S, 3, dtype=torch.int32, device=dev)
        act = torch.empty(E, S, 7, dtype=torch.uint8, device=dev)
        lp, v = torch.empty(E, device=dev), torch.empty(E, device=dev)
        al = torch.zeros(E, stride, dtype=torch.int32).pin_memory()
        st = MbkActStep()
        st.code_list, st.act_list, st.list_stride = rows.data_ptr(), al.data_ptr(), stride
        st.obs, st.mask, st.action, st.logp, st.value = (o.data_ptr(), mk.data_ptr(),
                                                         act.data_ptr(), lp.data_ptr(),
                                                         v.data_ptr())
        args = (ctypes.addressof(ws.struct), ctypes.addressof(st))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        tot = 0.0
        for i in range(steps + 3):
            st.step = i
            ev[0].record()
            N.check(k.mbk_act_step(*args, N.stream_ptr()), "act_step")
            ev[1].record()
            torch.cuda.synchronize()
            if i >= 3:
                tot += ev[0].elapsed_time(ev[1])
        active = float((mk != 0).any(-1).float().mean())
        out.append({"what": "policy_step", "target_active": f,
                    "active_frac": round(active, 4), "us_per_step": round(1e3 * tot / steps, 1),
                    "E": E})
        print(json.dumps(out[-1]), flush=True)
    return out


def cpu_sweep(E: int, steps: int) -> list[dict]:
    """env step cost (uniform-random agent, real games) binned by the active share"""
    from calibrate_env import uniform_legal

    from microbeast_amd import _native as N
    rt = N.runtime()
    env = rt.VecEnv(16, E, 2000, 3, [0, 0, 0, 1, 2, 3])
    obs = torch.zeros(E, S, dtype=torch.int32)
    mask = torch.zeros(E, S, 3, dtype=torch.int32)
    env.reset(obs.data_ptr(), mask.data_ptr())
    rew, done = torch.zeros(E), torch.zeros(E, dtype=torch.uint8)
    rng = np.random.default_rng(3)
    bins = {}
    for _ in range(steps):
        m = mask.numpy()
        af = float((m != 0).any(-1).mean())
        a = torch.from_numpy(uniform_legal(m, rng))
        t0 = time.perf_counter()
        env.step(a.data_ptr(), obs.data_ptr(), mask.data_ptr(), rew.data_ptr(), done.data_ptr())
        dt = time.perf_counter() - t0
        b = 0.005 if af < 0.0125 else 0.02 if af < 0.035 else 0.05
        n, s_ = bins.get(b, (0, 0.0))
        bins[b] = (n + 1, s_ + dt)
    out = []
    for b in sorted(bins):
        n, s_ = bins[b]
        out.append({"what": "env_step_cpu", "active_bin": b, "steps": n,
                    "us_per_env_step": round(1e6 * s_ / n / E, 3)})
        print(json.dumps(out[-1]), flush=True)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=8192)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--cpu_envs", type=int, default=256)
    p.add_argument("--cpu_steps", type=int, default=1500)
    p.add_argument("--cpu_only", action="store_true")
    a = p.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if not a.cpu_only:
        gpu_sweep(a.envs, (0.005, 0.02, 0.05), a.steps)
    cpu_sweep(a.cpu_envs, a.cpu_steps)


if __name__ == "__main__":
    main()
