"""Relu-gate flips of every residual conv0 output against the fp32 oracle, HIP vs torch-bf16
(the parity test's batch, tests/test_gpu_learner_parity.py): how many signs differ, at what
|u_ref|, and each path's relative error of u itself.

    python tools/dbg/gate_flips.py [--S 16]  (GPU)
"""
import argparse
import copy
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import engine_batches  # noqa: E402

from microbeast_amd.learner import Learner, LearnerHParams  # noqa: E402
from microbeast_amd.models.agent import Agent  # noqa: E402
from microbeast_amd.ops import encoder as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--S", type=int, default=16)
    a = ap.parse_args()
    cuda = torch.device("cuda", 0)
    S = a.S
    b = engine_batches(cuda, S, 2, groups=4, envs=64, T=8, seed=S)[1]
    torch.manual_seed(7)
    base = Agent((S, S, 27))
    with torch.no_grad():
        base.actor.weight.normal_(0, 0.02)
        base.actor.bias.normal_(0, 0.02)
    hip, ref, bf = copy.deepcopy(base), copy.deepcopy(base), copy.deepcopy(base)
    ref.hip_kernels = False
    ref.compute_dtype = torch.float32
    bf.hip_kernels = False
    caps = {"ref": {}, "bf": {}, "hip": {}}
    for name, m in (("ref", ref), ("bf", bf)):
        for si in range(3):
            for bi in (0, 1):
                blk = getattr(m.network[si], f"res_block{bi}")
                blk.conv0.register_forward_hook(
                    lambda mod, i, o, k=(si, bi), d=caps[name]: d.__setitem__(k, o.detach().double().cpu()))
                blk.register_forward_pre_hook(
                    lambda mod, i, k=(si, bi), d=caps[name]: d.__setitem__(("x",) + k, i[0].detach().double().cpu()))
    orig = E.HipEncoder.backward

    def bwd(self, g, saved, params):
        for s in range(len(saved) // 6):
            _x, _pidx, p, u0, y0, u1 = saved[6 * s:6 * s + 6]
            caps["hip"][(s, 0)] = u0.detach().double().cpu().permute(0, 3, 1, 2)
            caps["hip"][(s, 1)] = u1.detach().double().cpu().permute(0, 3, 1, 2)
            caps["hip"][("x", s, 0)] = p.detach().double().cpu().permute(0, 3, 1, 2)
            caps["hip"][("x", s, 1)] = y0.detach().double().cpu().permute(0, 3, 1, 2)
        return orig(self, g, saved, params)

    E.HipEncoder.backward = bwd
    Lh = Learner(hip, LearnerHParams(), cuda)
    Lb = Learner(bf, LearnerHParams(), cuda)
    Lr = Learner(ref, LearnerHParams(), torch.device("cpu"))
    Lh.learn(b)
    Lb.learn(b)
    torch.cuda.synchronize()
    Lr.learn({k: v.cpu() for k, v in b.items()})
    rel = lambda x, y: float((x - y).norm() / (y.norm() + 1e-300))  # noqa: E731
    for si in range(3):
        for bi in (0, 1):
            ur = caps["ref"][(si, bi)]
            n = ur.shape[0]
            xr = caps["ref"][("x", si, bi)]
            line = [f"stage {si} block {bi}: |u_ref| median {float(ur.abs().median()):.3e}"]
            for path in ("bf", "hip"):
                u = caps[path][(si, bi)][:n]
                x = caps[path][("x", si, bi)][:n]
                flip = (u > 0) != (ur > 0)
                nf = int(flip.sum())
                med = float(ur[flip].abs().median()) if nf else 0.0
                line.append(f"{path}: u rel {rel(u, ur):.2e} x rel {rel(x, xr):.2e} flips {nf} "
                            f"(|u_ref| median {med:.2e}, zeros in u {int((u == 0).sum())} "
                            f"vs ref {int((ur == 0).sum())})")
            print("\n    ".join(line), flush=True)


if __name__ == "__main__":
    main()
