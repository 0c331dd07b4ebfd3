"""The shifted-row GEMM (gemm.hip mbk_gemm_nt_taps) and shifted split-K weight gradient
(fc.hip mbk_fc_wgrad_taps) behind GridNet's convs, on the GPU, vs fp32 F.conv2d /
F.conv_transpose2d on the same bf16-rounded operands (fwd + all grads)."""
import pytest
import torch

from test_gridconv import _check, _ref_conv, _ref_convt
from microbeast_amd.ops import gridconv as gc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cin,cout,b,hw,relu", [(27, 32, 40, 16, True), (64, 128, 64, 4, True),
                                                (256, 64, 9, 3, False)])
def test_gpu_conv3x3(cin, cout, b, hw, relu):
    torch.manual_seed(0)
    x = torch.randn(b, hw, hw, cin)
    w = torch.randn(cout, cin, 3, 3) * 0.05
    bias = torch.randn(cout) * 0.1
    _check(gc.conv3x3, _ref_conv, x, w, bias, relu, "cuda", 2e-2)


@pytest.mark.parametrize("cin,cout,b,hw,relu", [(256, 128, 50, 1, True), (64, 32, 33, 4, True),
                                                (32, 78, 20, 8, False)])
def test_gpu_conv_transpose(cin, cout, b, hw, relu):
    torch.manual_seed(0)
    x = torch.randn(b, hw, hw, cin)
    w = torch.randn(cin, cout, 3, 3) * 0.05
    bias = torch.randn(cout) * 0.1
    _check(gc.conv_transpose3x3s2, _ref_convt, x, w, bias, relu, "cuda", 2e-2)


def test_gpu_taps_gemm_matches_emulation():
    torch.manual_seed(0)
    M, tk, n = 1000, 64, 96
    bases = [torch.randn(M, tk, device="cuda").to(torch.bfloat16) for _ in range(3)]
    shifts = [-37, 0, 300]
    b = torch.randn(n, 3 * tk, device="cuda").to(torch.bfloat16)
    bias = torch.randn(n, device="cuda")
    got = gc.taps_gemm(bases, shifts, b, bias, relu=True, out_dtype=torch.float32)
    want = gc._taps_gemm_ref(bases, shifts, b, bias, True, torch.float32)
    torch.testing.assert_close(got, want, rtol=1e-3, atol=1e-3)
    g = torch.randn(M, 40, device="cuda").to(torch.bfloat16)
    gw = gc.taps_wgrad(g, bases[0], shifts)
    torch.testing.assert_close(gw, gc._taps_wgrad_ref(g, bases[0], shifts), rtol=1e-3, atol=2e-2)
