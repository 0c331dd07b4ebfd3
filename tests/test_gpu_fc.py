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


@pytest.mark.parametrize("n,i", [(266240, 128), (5037, 128), (9000, 32), (70001, 64), (100, 128)])
def test_fc_wgrad_wide_weight_and_bias(cuda, n, i):
    """One-pass dW = g^T relu(x), db = g^T 1 (fc_wgrad_wide_kernel, the IMPALA tail's FC)
    vs fp32 PyTorch, including partial last stages and fewer rows than workgroups."""
    from microbeast_amd import _native as N
    k = N.kernels()
    o = 256
    torch.manual_seed(n + i)
    g = torch.randn(n, o, device=cuda).bfloat16()
    x = torch.randn(n, i, device=cuda).bfloat16()
    parts = k.mbk_fc_wgrad_wide_parts(n, o, i)
    assert parts > 0
    scratch = torch.empty((parts + (parts + 31) // 32) * (o * i + o), device=cuda)
    dw = torch.empty(o, i, device=cuda)
    db = torch.empty(o, device=cuda)
    N.check(k.mbk_fc_wgrad_wide(g.data_ptr(), x.data_ptr(), n, o, i, 1, scratch.data_ptr(),
                                parts, dw.data_ptr(), db.data_ptr(), N.stream_ptr()),
            "fc_wgrad_wide")
    ref_w = g.float().t() @ torch.relu(x.float())
    ref_b = g.float().sum(0)
    assert ((dw - ref_w).norm() / ref_w.norm()).item() < 1e-5
    assert ((db - ref_b).norm() / ref_b.norm()).item() < 1e-5
    assert k.mbk_fc_wgrad_wide_parts(n, o, 288) == 0  # uncovered shapes fall back
