"""Hand-written MFMA GEMM (gemm.hip) vs fp32 torch, forward and autograd."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(1000, 256, 128), (257, 77, 40), (5, 1, 256), (4096, 384, 288),
                                   (130, 130, 8), (1000, 32, 64), (700, 64, 96), (513, 20, 32),
                                   (300, 40, 288)])
def test_gemm_nt_forward(cuda, M, N, K):
    from microbeast_amd.ops.gemm import gemm_nt_raw
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    bias = torch.randn(N, device=cuda)
    ref = a.float() @ b.float().t() + bias
    y = gemm_nt_raw(a, b, bias)
    assert _rel(y, ref) < 5e-3
    yr = gemm_nt_raw(a, b, bias, relu=True)
    assert _rel(yr, ref.clamp_min(0)) < 5e-3
    # fp32 output, accumulate into C
    c = torch.ones(M, N, device=cuda)
    gemm_nt_raw(a, b, None, out=c, accumulate=True)
    assert _rel(c, a.float() @ b.float().t() + 1) < 5e-3
    # strided A rows (a view into a wider buffer)
    wide = torch.randn(M, K + 16, device=cuda).bfloat16()
    y2 = gemm_nt_raw(wide[:, :K], b)
    assert _rel(y2, wide[:, :K].float() @ b.float().t()) < 5e-3


def test_gemm_nt_autograd(cuda):
    from microbeast_amd.ops.gemm import gemm_nt
    torch.manual_seed(0)
    a = torch.randn(3000, 64, device=cuda).bfloat16().requires_grad_(True)
    w = (torch.randn(96, 64, device=cuda) * 0.1).requires_grad_(True)
    bias = torch.randn(96, device=cuda).requires_grad_(True)
    y = gemm_nt(a, w, bias, relu=True)
    r = torch.randn_like(y.float())
    (y.float() * r).sum().backward()
    ar = a.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = bias.detach().clone().requires_grad_(True)
    yr = torch.relu(ar @ wr.t() + br)
    (yr * r).sum().backward()
    assert _rel(y, yr) < 5e-3
    assert w.grad.dtype == torch.float32
    assert _rel(a.grad, ar.grad) < 1e-2
    assert _rel(w.grad, wr.grad) < 1e-2
    assert _rel(bias.grad, br.grad) < 1e-2


@pytest.mark.parametrize("M,N,K", [(1000, 128, 256), (300, 40, 64), (129, 77, 32)])
def test_gemm_nt_mask_matches_torch(cuda, M, N, K):
    """mbk_gemm_nt_mask (relu-backward mask in the epilogue; N % 8 == 0 takes the LDS-staged
    16-byte epilogue, N = 77 the per-element one) vs fp32 torch."""
    from microbeast_amd import _native as Nn
    torch.manual_seed(M + N)
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    mask = torch.randn(M, N, device=cuda).bfloat16()
    c = torch.full((M, N), 7.0, device=cuda).bfloat16()
    Nn.check(Nn.kernels().mbk_gemm_nt_mask(a.data_ptr(), b.data_ptr(), c.data_ptr(), None, M, N,
                                           K, K, K, N, 0, 1, mask.data_ptr(), Nn.stream_ptr()),
             "gemm_nt_mask")
    ref = (a.float() @ b.float().t()) * (mask.float() > 0)
    assert _rel(c, ref) < 5e-3
    assert bool(((mask.float() > 0) | (c.float() == 0)).all())
