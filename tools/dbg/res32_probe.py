"""Debug: delta inputs through res_bwd32 to read off the wgrad operand mapping."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from microbeast_amd.ops.encoder import HipEncoder

dev = torch.device("cuda", 0)
enc = HipEncoder(16, 16, 27, device=dev)
L0, L1 = enc.layers[6], enc.layers[7]
ws = [torch.zeros(c.cout, c.cin_real, 3, 3, device=dev) for c in enc.layers]
enc.pack([w.contiguous() for w in ws], with_bwd=True)
n = 8
for (py, px, co, ci) in ((1, 1, 0, 0), (1, 1, 5, 0), (1, 1, 0, 5), (2, 1, 3, 7), (1, 1, 20, 0),
                         (1, 1, 0, 20)):
    x = torch.zeros(n, 4, 4, 32, device=dev).bfloat16()
    u = torch.zeros(n, 4, 4, 32, device=dev).bfloat16()
    g = torch.zeros(n, 4, 4, 32, device=dev).bfloat16()
    g[0, py, px, co] = 1.0
    u[0, py, px, ci] = 1.0
    dw1 = torch.zeros(32, 32, 3, 3, device=dev); db1 = torch.zeros(32, device=dev)
    dw0 = torch.zeros(32, 32, 3, 3, device=dev); db0 = torch.zeros(32, device=dev)
    enc._res_bwd32(L0, L1, x, u, g, dw1, db1, dw0, db0)
    torch.cuda.synchronize()
    nz = dw1.nonzero().tolist()
    print(f"pix ({py},{px}) co {co} ci {ci}: expect [{co}, {ci}, 1, 1]; got", nz[:12],
          [float(dw1[tuple(i)]) for i in nz[:12]])
