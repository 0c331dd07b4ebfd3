"""Shifted-row (implicit im2col) GridNet convolutions (ops/gridconv.py): the tap / shift
index maths, forward and every gradient, against F.conv2d / F.conv_transpose2d in fp32.
On CPU the launchers run their torch emulation; tests/test_gpu_gridconv.py runs the same
checks on the HIP kernels."""
import pytest
import torch
import torch.nn.functional as F

from microbeast_amd.ops import gridconv as gc


def _ref_conv(x, w, b, relu):
    y = F.conv2d(x.permute(0, 3, 1, 2), w, b, padding=1)
    return (F.relu(y) if relu else y).permute(0, 2, 3, 1)


def _ref_convt(x, w, b, relu):
    y = F.conv_transpose2d(x.permute(0, 3, 1, 2), w, b, stride=2, padding=1, output_padding=1)
    return (F.relu(y) if relu else y).permute(0, 2, 3, 1)


def _check(fn, ref, x, w, b, relu, device, tol):
    torch.manual_seed(1)
    xb = x.to(device, torch.bfloat16).requires_grad_(True)
    wd = w.to(device).requires_grad_(True)
    bd = b.to(device).requires_grad_(True)
    y = fn(xb, wd, bd, relu)
    gy = torch.randn(y.shape, device=device)
    (y.float() * gy).sum().backward()
    # fp32 reference on the same bf16-rounded operands
    xr = xb.detach().float().requires_grad_(True)
    wr = wd.detach().to(torch.bfloat16).float().requires_grad_(True)
    br = bd.detach().clone().requires_grad_(True)
    yr = ref(xr, wr, br, relu)
    (yr * gy).sum().backward()
    s = float(yr.abs().max()) + 1e-6
    assert float((y.float() - yr).abs().max()) / s < tol
    for got, want in ((xb.grad, xr.grad), (wd.grad, wr.grad), (bd.grad, br.grad)):
        assert got.shape == want.shape
        m = float(want.abs().max()) + 1e-6
        assert float((got.float() - want).abs().max()) / m < tol


@pytest.mark.parametrize("cin,cout,hw,relu", [(27, 32, 6, True), (32, 64, 4, False),
                                              (64, 40, 3, True)])
def test_conv3x3_matches_conv2d(cin, cout, hw, relu):
    torch.manual_seed(0)
    x = torch.randn(3, hw, hw + 1, cin)
    w = torch.randn(cout, cin, 3, 3) * 0.1
    b = torch.randn(cout) * 0.1
    _check(gc.conv3x3, _ref_conv, x, w, b, relu, "cpu", 2e-2)


@pytest.mark.parametrize("cin,cout,hw,relu", [(64, 32, 2, True), (32, 78, 3, False),
                                              (40, 16, 1, True)])
def test_conv_transpose_matches(cin, cout, hw, relu):
    torch.manual_seed(0)
    x = torch.randn(2, hw, hw + 1, cin)
    w = torch.randn(cin, cout, 3, 3) * 0.1
    b = torch.randn(cout) * 0.1
    _check(gc.conv_transpose3x3s2, _ref_convt, x, w, b, relu, "cpu", 2e-2)


def test_phase_taps_cover_kernel_once():
    taps = [(ky, kx) for _, _, t in gc._phase_taps(5) for ky, kx, _ in t]
    assert sorted(taps) == [(ky, kx) for ky in range(3) for kx in range(3)]
