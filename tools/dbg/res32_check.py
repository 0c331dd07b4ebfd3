"""Debug: one 32-channel residual block backward through resblock.hip res_bwd32 vs fp32
autograd; prints per-(tap, co-block, ci-block) errors of dW1 / dW0 and dx / bias errors."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import torch.nn.functional as Fn

from microbeast_amd.ops.encoder import ConvLayer, HipEncoder

dev = torch.device("cuda", 0)
torch.manual_seed(0)
H = W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
enc = HipEncoder(16, 16, 27, device=dev)
L0, L1 = enc.layers[6], enc.layers[7]
assert L0.cin == 32 and L0.H == 4
L0 = ConvLayer(32, 32, 32, H, W, False, True, False, L0.w_off, L0.wb_off)
L1 = ConvLayer(32, 32, 32, H, W, False, True, False, L1.w_off, L1.wb_off)
ws = [torch.randn(c.cout, c.cin_real, 3, 3, device=dev) * 0.1 for c in enc.layers]
enc.pack([w.contiguous() for w in ws], with_bwd=True)
w0, w1 = ws[6], ws[7]
x = torch.randn(n, H, W, 32, device=dev).bfloat16()
u = torch.randn(n, H, W, 32, device=dev).bfloat16()
g = torch.randn(n, H, W, 32, device=dev).bfloat16()
dw1 = torch.zeros(32, 32, 3, 3, device=dev); db1 = torch.zeros(32, device=dev)
dw0 = torch.zeros(32, 32, 3, 3, device=dev); db0 = torch.zeros(32, device=dev)
dx = enc._res_bwd32(L0, L1, x, u, g, dw1, db1, dw0, db0)
torch.cuda.synchronize()
# reference: u given (not recomputed): du = conv1^T(g) * [u > 0]; dx = conv0^T(du) * [x>0] + g
nchw = lambda t: t.float().permute(0, 3, 1, 2)
ru = torch.relu(nchw(u)).requires_grad_(True)
y1 = Fn.conv2d(ru, w1, padding=1)
rdw1, = torch.autograd.grad((y1 * nchw(g)).sum(), [w1.requires_grad_(True)]) if False else (None,)
w1r = w1.clone().requires_grad_(True)
y1 = Fn.conv2d(ru, w1r, padding=1)
gw1, gru = torch.autograd.grad((y1 * nchw(g)).sum(), [w1r, ru])
du = gru * (nchw(u) > 0)
du_b = du.bfloat16().float()
rx = torch.relu(nchw(x)).requires_grad_(True)
w0r = w0.clone().requires_grad_(True)
y0 = Fn.conv2d(rx, w0r, padding=1)
gw0, grx = torch.autograd.grad((y0 * du_b).sum(), [w0r, rx])
dxr = grx * (nchw(x) > 0) + nchw(g)


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


print("dx rel", rel(nchw(dx), dxr))
print("db1 rel", rel(db1, nchw(g).sum((0, 2, 3))), "db0 rel", rel(db0, du_b.sum((0, 2, 3))))
for name, a, b in (("dW1", dw1, gw1), ("dW0", dw0, gw0)):
    print(name, "rel", rel(a, b))
    for t in range(9):
        row = []
        for cb in range(2):
            for cib in range(2):
                aa = a[cb * 16:cb * 16 + 16, cib * 16:cib * 16 + 16, t // 3, t % 3]
                bb = b[cb * 16:cb * 16 + 16, cib * 16:cib * 16 + 16, t // 3, t % 3]
                row.append(f"{rel(aa, bb):.2e}")
        print("  tap", t, " ".join(row))
