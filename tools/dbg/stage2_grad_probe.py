"""Where does the HIP learner's stage-2 block-1 conv0 gradient leave the fp32 reference?
Same batch as tests/test_gpu_learner_parity.py (S=16, 4 x 64 envs); captures the trunk
output y, its gradient g, and the saved stage-2 activations on both paths."""
import copy
import sys

import torch

sys.path.insert(0, "tests")
from helpers import engine_batches  # noqa: E402

from microbeast_amd.learner import Learner, LearnerHParams  # noqa: E402
from microbeast_amd.models.agent import Agent  # noqa: E402
from microbeast_amd.ops import encoder as E  # noqa: E402

cuda = torch.device("cuda", 0)
S = 16
b = engine_batches(cuda, S, 2, groups=4, envs=64, T=8, seed=S)[1]
torch.manual_seed(7)
base = Agent((S, S, 27))
with torch.no_grad():
    base.actor.weight.normal_(0, 0.02)
    base.actor.bias.normal_(0, 0.02)
hip, ref = copy.deepcopy(base), copy.deepcopy(base)
ref.hip_kernels = False
ref.compute_dtype = torch.float32
cap = {}
orig_bwd = E.HipEncoder.backward


def bwd(self, g, saved, params):
    cap["g_hip"] = g.float().clone()
    cap["saved_hip"] = [t.clone() for t in saved]
    return orig_bwd(self, g, saved, params)


E.HipEncoder.backward = bwd
st2 = ref.network[2]
hooks = {}


def fwd_hook(name):
    def h(mod, inp, out):
        hooks[name] = out
        out.retain_grad()
    return h


st2.res_block1.conv0.register_forward_hook(fwd_hook("u1"))
st2.register_forward_hook(fwd_hook("y"))
Lh = Learner(hip, LearnerHParams(), cuda)
Lr = Learner(ref, LearnerHParams(), torch.device("cpu"))
Lh.learn(b)
torch.cuda.synchronize()
Lr.learn({k: v.cpu() for k, v in b.items()})
gh = cap["g_hip"].cpu()                         # NHWC [n, 2, 2, 32]
gr = hooks["y"].grad.permute(0, 2, 3, 1)        # NCHW -> NHWC
yr = hooks["y"].detach().permute(0, 2, 3, 1)
n = gr.shape[0]
gh = gh[:n]
rel = lambda a, c: float((a - c).norm() / (c.norm() + 1e-30))  # noqa: E731
print("g  rel", rel(gh, gr), "shape", tuple(gh.shape), tuple(gr.shape))
sv = cap["saved_hip"]
u1h = sv[6 * 2 + 5].float().cpu()[:n]           # stage 2: x, pidx, p, u0, y0, u1
u1r = hooks["u1"].detach().permute(0, 2, 3, 1)
print("u1 rel", rel(u1h, u1r), " mask agreement", float(((u1h > 0) == (u1r > 0)).float().mean()))
# per pixel position / channel error of g
for py in range(2):
    for px in range(2):
        print(f"g pixel ({py},{px}) rel", rel(gh[:, py, px], gr[:, py, px]))
dw_h = Lh.flat.grad.cpu()
