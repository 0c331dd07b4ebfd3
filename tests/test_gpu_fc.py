"""Split-K FC weight gradient (fc.hip) vs the fp32 PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,o,i", [(266240, 256, 128), (5037, 256, 128), (70001, 1, 256),
                                   (9000, 256, 32), (20000, 256, 288)])
def test_fc_weight_grad_matches_fp32(cuda, n, o, i):
    from microbeast_amd.ops.linear import weight_grad
    torch.manual_seed(n)
    g = torch.randn(n, o, device=cuda).bfloat16()
    x = torch.randn(n, i, device=cuda).bfloat16()
    out = weight_grad(g, x)
    ref = g.float().t() @ x.float()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 1e-5, rel


def test_linear_autograd_matches_reference_layer(cuda):
    from microbeast_amd.ops.linear import linear
    torch.manual_seed(0)
    lin = torch.nn.Linear(128, 256).to(cuda)
    y = torch.randn(9000, 2, 2, 32, device=cuda).bfloat16().requires_grad_(True)
    out = linear(y.reshape(9000, -1), lin, nhwc=(32, 2, 2))
    r = torch.randn_like(out)
    (out.float() * r).sum().backward()
    gw, gb, gy = lin.weight.grad.clone(), lin.bias.grad.clone(), y.grad.clone()
    # fp32 reference on the same bf16-rounded operands (the grad of the cast itself
    # would round the reference gradient to bf16)
    wr = lin.weight.detach().bfloat16().float().requires_grad_(True)
    br = lin.bias.detach().clone().requires_grad_(True)
    yr = y.detach().float().permute(0, 3, 1, 2).reshape(9000, -1).requires_grad_(True)
    (torch.nn.functional.linear(yr, wr, br) * r.float()).sum().backward()
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(gw, wr.grad) < 1e-3
    assert rel(gb, br.grad) < 1e-3
    assert rel(gy.float().permute(0, 3, 1, 2).reshape(9000, -1), yr.grad) < 1e-2
