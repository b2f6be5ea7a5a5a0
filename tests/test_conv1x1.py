"""1x1 convolutions as NHWC GEMMs with the residual-gradient sum folded into the dgrad GEMM
(ops/conv1x1.py): forward, input gradient (both branches) and weight gradient against
nn.Conv2d + autograd's own branch sum, on CPU fp32 for every GEMM / MIOpen-path choice."""
import pytest
import torch

from cloudtik_amd.ops import conv1x1 as C1


def _data(N=2, C=16, H=5, co=24, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, H, H, generator=g).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(co, C, 1, 1, generator=g) * 0.2).contiguous(memory_format=torch.channels_last)
    return x, w


@pytest.mark.parametrize("fwd_min,dgrad_min", [(1, 1), (10 ** 6, 10 ** 6), (1, 10 ** 6)])
@pytest.mark.parametrize("keep", [False, True])
def test_conv1x1_matches_conv2d(monkeypatch, fwd_min, dgrad_min, keep):
    monkeypatch.setattr(C1, "FWD_GEMM_MIN_CIN", fwd_min)
    monkeypatch.setattr(C1, "DGRAD_GEMM_MIN_CIN", dgrad_min)
    x, w = _data()
    s = torch.randn(1, 16, 1, 1)          # the other branch: a channel scale of x

    def ref_loss(x, w):
        y = torch.nn.functional.conv2d(x, w)
        other = (x * s).sum() if keep else 0.0
        return (y * torch.arange(y.numel()).view_as(y).cos()).sum() + other

    x1, w1 = x.clone().requires_grad_(), w.clone().requires_grad_()
    ref_loss(x1, w1).backward()

    x2, w2 = x.clone().requires_grad_(), w.clone().requires_grad_()
    out = C1._Conv1x1Fn.apply(x2, w2, keep)
    if keep:
        y, xa = out
        other = (xa * s).sum()
    else:
        y, other = out, 0.0
    assert y.is_contiguous(memory_format=torch.channels_last)
    ((y * torch.arange(y.numel()).view_as(y).cos()).sum() + other).backward()
    torch.testing.assert_close(y, torch.nn.functional.conv2d(x, w), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x2.grad, x1.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(w2.grad, w1.grad, rtol=1e-5, atol=1e-5)


def test_alias_gradient_is_accumulated_in_place(monkeypatch):
    """The other branch's fresh NHWC gradient is the buffer the dgrad GEMM accumulates into
    (no extra tensor): the input gradient comes out as that very storage."""
    monkeypatch.setattr(C1, "DGRAD_GEMM_MIN_CIN", 1)
    x, w = _data(C=8, co=8)
    seen = {}

    class Other(torch.autograd.Function):
        @staticmethod
        def forward(ctx, t):
            return t * 2

        @staticmethod
        def backward(ctx, g):
            d = (g * 2).contiguous(memory_format=torch.channels_last)
            seen["ptr"] = d.data_ptr()
            return d

    xr = x.clone().requires_grad_()
    y, xa = C1._Conv1x1Fn.apply(xr, w, True)
    (y.sum() + Other.apply(xa).sum()).backward()
    ref = torch.nn.functional.conv2d(x.clone().requires_grad_(), w)
    xr2 = x.clone().requires_grad_()
    (torch.nn.functional.conv2d(xr2, w).sum() + (xr2 * 2).sum()).backward()
    torch.testing.assert_close(xr.grad, xr2.grad)
    assert xr.grad.data_ptr() == seen["ptr"] and ref is not None


def test_bottleneck_uses_alias_and_matches_plain_convs():
    """The model path: CPU falls back to nn.Conv2d, so the bottleneck output is unchanged."""
    from cloudtik_amd.models.resnet import Bottleneck
    torch.manual_seed(0)
    b = Bottleneck(16, 4, downsample=True, dtype=torch.float32)
    x = torch.randn(2, 16, 6, 6)
    ref = b.bn3(b.conv3(b.bn2(b.conv2(b.bn1(b.conv1(x))))), residual=b.down_bn(b.down(x)))
    torch.testing.assert_close(b(x), ref)
    assert not C1.conv1x1_eligible(x, b.conv1)        # CPU / fp32: stock conv


def test_conv3x3_dgrad_as_forward_conv():
    """3x3 stride-1 dgrad issued as conv2d(dY, flip(W)^T, pad 1) equals autograd's."""
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 6, 7, 7, generator=g).contiguous(memory_format=torch.channels_last)
    w = torch.randn(5, 6, 3, 3, generator=g).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(2, 5, 7, 7, generator=g)
    x1, w1 = x.clone().requires_grad_(), w.clone().requires_grad_()
    torch.nn.functional.conv2d(x1, w1, padding=1).backward(dy)
    x2, w2 = x.clone().requires_grad_(), w.clone().requires_grad_()
    y = C1._Conv3x3Fn.apply(x2, w2)
    y.backward(dy)
    torch.testing.assert_close(x2.grad, x1.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(w2.grad, w1.grad, rtol=1e-5, atol=1e-5)
