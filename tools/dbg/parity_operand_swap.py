"""Root-cause probe for the learner-parity outlier: which operand makes the
HIP gradient of network.2.res_block1.conv0 (stage 2, 2x2 maps) leave the fp32 oracle by ~8x
the torch-bf16 floor?

That gradient is a function of three tensors only:
    dW = wgrad( relu(y0), du1 ),   du1 = dgrad_conv1( g ) * [u1 > 0]
y0 = the block's input, u1 = its conv0 output, g = the stage output's gradient. The same
batch as tests/test_gpu_learner_parity.py (S = 16) runs through three learners -- fp32 torch
(CPU, the oracle), torch under bf16 autocast (GPU, the floor) and the HIP path -- capturing
(y0, u1, g) from each. dW is then recomputed in fp64 for every operand mix, e.g. (y0, u1) of
the oracle with g of the HIP path: the operand whose swap carries the error is the cause.

    python tools/dbg/parity_operand_swap.py  (GPU)
"""
import copy
import itertools
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import engine_batches  # noqa: E402

from microbeast_amd.learner import Learner, LearnerHParams  # noqa: E402
from microbeast_amd.models.agent import Agent  # noqa: E402
from microbeast_amd.ops import encoder as E  # noqa: E402

cuda = torch.device("cuda", 0)
S = 16
LAYER = "network.2.res_block1.conv0.weight"


def torch_capture(model):
    """hooks on stage 2: y0 (res_block1 input), u1 (its conv0 output), g (stage output grad)"""
    st2 = model.network[2]
    cap = {}

    def pre(mod, inp):
        cap["y0"] = inp[0].detach()

    def u1(mod, inp, out):
        cap["u1"] = out.detach()

    def y(mod, inp, out):
        out.register_hook(lambda gr: cap.__setitem__("g", gr.detach()))

    st2.res_block1.register_forward_pre_hook(pre)
    st2.res_block1.conv0.register_forward_hook(u1)
    st2.register_forward_hook(y)
    return cap


def nchw(t):  # NHWC -> NCHW, fp64 CPU
    return t.detach().double().cpu().permute(0, 3, 1, 2).contiguous()


def dw(y0, u1, g, w1):
    """fp64 weight gradient of conv0 from the three operands (NCHW)"""
    du1 = torch.nn.grad.conv2d_input(u1.shape, w1, g, padding=1) * (u1 > 0)
    return torch.nn.grad.conv2d_weight(F.relu(y0), (32, 32, 3, 3), du1, padding=1)


def main():
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
    cr, cb = torch_capture(ref), torch_capture(bf)
    ch = {}
    orig_bwd = E.HipEncoder.backward

    def bwd(self, g, saved, params):
        ch["g"] = g.float().clone()
        x, pidx, p, u0, y0, u1 = saved[12:18]
        ch["y0"], ch["u1"] = y0.float().clone(), u1.float().clone()
        return orig_bwd(self, g, saved, params)

    E.HipEncoder.backward = bwd
    Lh = Learner(hip, LearnerHParams(), cuda)
    Lr = Learner(ref, LearnerHParams(), torch.device("cpu"))
    Lb = Learner(bf, LearnerHParams(), cuda)
    Lh.learn(b)
    Lb.learn(b)
    torch.cuda.synchronize()
    Lr.learn({k: v.cpu() for k, v in b.items()})
    n = cr["g"].shape[0]
    ops = {
        "ref": {k: cr[k].double().cpu() for k in ("y0", "u1", "g")},
        "bf16": {k: cb[k].double().cpu() for k in ("y0", "u1", "g")},
        "hip": {k: nchw(ch[k][:n]) for k in ("y0", "u1", "g")},
    }
    w1 = ref.network[2].res_block1.conv1.weight.detach().double()
    rel = lambda a, c: float((a - c).norm() / (c.norm() + 1e-300))  # noqa: E731
    want = dw(**ops["ref"], w1=w1)
    for name, off, cnt, _ in Lr.flat.slices:
        if name == LAYER:
            gh = Lh.flat.grad.cpu()[off:off + cnt].double().view_as(want)
            gr = Lr.flat.grad[off:off + cnt].double().view_as(want)
            gb = Lb.flat.grad.cpu()[off:off + cnt].double().view_as(want)
    print(f"learner grads vs oracle: hip rel {rel(gh, gr):.4f}  torch-bf16 rel {rel(gb, gr):.4f}"
          f"  (oracle recomputed from its operands: rel {rel(want, gr):.2e})")
    for path in ("bf16", "hip"):
        for k in ("y0", "u1", "g"):
            a, c = ops[path][k], ops["ref"][k]
            extra = ""
            if k == "u1":
                extra = f" sign agreement {float(((a > 0) == (c > 0)).double().mean()):.5f}"
            print(f"  {path:5s} {k:3s} rel {rel(a, c):.4f}{extra}")
    print("dW recomputed from mixed operands (rel to the oracle):")
    for src in itertools.product(("ref", "bf16", "hip"), repeat=3):
        if len(set(src) - {"ref"}) > 1:
            continue
        y0, u1, g = (ops[s_][k] for s_, k in zip(src, ("y0", "u1", "g")))
        print(f"  y0={src[0]:5s} u1={src[1]:5s} g={src[2]:5s}  rel {rel(dw(y0, u1, g, w1), want):.4f}")
    # the mask flips: where, how big are u1 there, how much du do they gate?
    du_ref = torch.nn.grad.conv2d_input(ops["ref"]["u1"].shape, w1, ops["ref"]["g"], padding=1)
    ur = ops["ref"]["u1"]
    for path in ("bf16", "hip"):
        uo = ops[path]["u1"]
        flip = (uo > 0) != (ur > 0)
        nf = int(flip.sum())
        imp = float(du_ref[flip].abs().sum() / du_ref.abs().sum())
        print(f"{path}: {nf} mask flips of {flip.numel()}; share of |du| they gate {imp:.4f}")
        if nf:
            print(f"  |u1_ref| at flips: median {float(ur[flip].abs().median()):.3e} max "
                  f"{float(ur[flip].abs().max()):.3e}; |u1_{path}| median "
                  f"{float(uo[flip].abs().median()):.3e}; zeros in u1_{path} at flips "
                  f"{int((uo[flip] == 0).sum())}; zeros overall {int((uo == 0).sum())} "
                  f"(ref {int((ur == 0).sum())})")
            print(f"  flips per channel {flip.sum((0, 2, 3)).tolist()}")
            print(f"  flips per pixel {flip.sum((0, 1)).flatten().tolist()}")
            print(f"  u1_ref > 0 at flips: {int((ur[flip] > 0).sum())}")
    # is u1_hip the conv of ITS OWN input? emulate conv0(relu(y0_hip)) in fp64 with the
    # bf16-rounded weights and fp32 bias, then round to bf16 like the kernel's epilogue
    c0 = ref.network[2].res_block1.conv0
    w0b = c0.weight.detach().bfloat16().double()
    emu = F.conv2d(F.relu(ops["hip"]["y0"]), w0b, c0.bias.detach().double(), padding=1)
    emu_b = emu.float().bfloat16().double()
    emu_r = F.conv2d(F.relu(ops["ref"]["y0"]), w0b, c0.bias.detach().double(), padding=1)
    emu_b16 = F.conv2d(F.relu(ops["bf16"]["y0"]), w0b, c0.bias.detach().double(), padding=1)
    print(f"sanity: u1_ref vs emulation on y0_ref {rel(ur, emu_r):.2e}; u1_bf16 vs emulation on "
          f"y0_bf16 {rel(ops['bf16']['u1'], emu_b16):.2e}; emulation(y0_hip) vs u1_ref "
          f"{rel(emu, ur):.2e}")
    # per frame: is the mismatch in a few frames (e.g. rows from another frame)?
    fe = (ops["hip"]["u1"] - emu).flatten(1).norm(dim=1) / (emu.flatten(1).norm(dim=1) + 1e-30)
    top = torch.argsort(fe, descending=True)[:8]
    print("frames with the largest u1_hip vs own-input error:",
          [(int(f), round(float(fe[f]), 4)) for f in top], "median", float(fe.median()))
    print(f"u1_hip vs fp64 emulation on its own input: rel {rel(ops['hip']['u1'], emu):.2e}, "
          f"bf16-rounded emu equal {float((emu_b == ops['hip']['u1']).double().mean()):.5f}, "
          f"sign flips vs emu {int(((emu > 0) != (ops['hip']['u1'] > 0)).sum())}")
    for path in ("bf16", "hip"):
        d = ops[path]["u1"] - ur
        print(f"{path}: per-channel mean(u1 - u1_ref) x1e5 "
              f"{[round(float(v) * 1e5, 2) for v in d.mean((0, 2, 3))]}")
        print(f"{path}: per-channel std(u1 - u1_ref) x1e5 "
              f"{[round(float(v) * 1e5, 2) for v in d.std((0, 2, 3))]}")
    print(f"|du_ref| per channel (mean x1e6): "
          f"{[round(float(v) * 1e6, 2) for v in du_ref.abs().mean((0, 2, 3))]}")
    print(f"|u1_ref| per channel (median x1e3): "
          f"{[round(float(v) * 1e3, 3) for v in ur.abs().median(3)[0].median(2)[0].median(0)[0]]}")
    # where in g: per pixel, and concentrated in few frames?
    dg = (ops["hip"]["g"] - ops["ref"]["g"]).flatten(1).norm(dim=1)
    gn = ops["ref"]["g"].flatten(1).norm(dim=1)
    top = torch.argsort(dg, descending=True)[:10]
    print("frames with the largest g error (err / |g_ref| / active cells):")
    act = (b["mask"].view(-1, S * S, 3) != 0).any(-1).sum(1).cpu()
    for f in top.tolist():
        print(f"  frame {f}: {float(dg[f]):.3e} / {float(gn[f]):.3e} / {int(act[f])}")
    dgb = (ops["bf16"]["g"] - ops["ref"]["g"]).flatten(1).norm(dim=1)
    print(f"share of g error in the top 1% frames: hip {float(dg.sort(descending=True)[0][:max(1, n // 100)].pow(2).sum() / dg.pow(2).sum()):.3f}"
          f" bf16 {float(dgb.sort(descending=True)[0][:max(1, n // 100)].pow(2).sum() / dgb.pow(2).sum()):.3f}")


if __name__ == "__main__":
    main()
