"""Stage-2 (2x2 map) dgrad with a relu mask, HIP vs fp32 torch on the same bf16 operands:
du = conv1^T(g) * [u > 0] for every 32-channel layer shape of the 16x16 trunk."""
import torch
import torch.nn.functional as F

from microbeast_amd.models.agent import Agent
from microbeast_amd.ops.encoder import encoder_params

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = Agent((16, 16, 27)).to(dev)
obs = torch.randint(0, 1 << 27, (4, 256), dtype=torch.int32, device=dev)
m.features(obs)
enc = m._hip_enc
params = [p.detach() for p in encoder_params(m.network, 3)]
ws = params[0::2]
enc.pack([w.contiguous() for w in ws], with_bwd=True)
for li in (6, 7, 8, 9, 11, 12, 13, 14):
    L = enc.layers[li]
    n = 512
    g = torch.randn(n, L.H, L.W, L.cout, device=dev).bfloat16()
    u = torch.randn(n, L.H, L.W, L.cin, device=dev).bfloat16()
    du = enc._fwd(L, g, None, mask_src=u, dgrad=True).float()
    wb = ws[li].bfloat16().float()
    gi = g.float().permute(0, 3, 1, 2)
    ref = F.conv_transpose2d(gi, wb, padding=1).permute(0, 2, 3, 1) * (u.float() > 0)
    rel = ((du - ref).norm() / ref.norm()).item()
    print(f"layer {li} {L.H}x{L.W} cin {L.cin} cout {L.cout}: rel {rel:.2e}")
