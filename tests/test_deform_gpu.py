"""Deformable conv / PS RoI pooling HIP kernels vs the fp32 PyTorch references (forward and
every gradient)."""
import pytest
import torch

from cloudtik_amd.ops.deform import (deform_conv2d, deform_conv2d_reference, deform_roi_pooling,
                                     deform_roi_pooling_reference)

pytestmark = pytest.mark.gpu
dev = torch.device("cuda", 0)


@pytest.mark.parametrize("modulated", [False, True])
@pytest.mark.parametrize("cfg", [dict(stride=1, padding=1, dilation=1, groups=1, dg=1),
                                 dict(stride=2, padding=2, dilation=2, groups=2, dg=2)])
def test_deform_conv_fwd_bwd(modulated, cfg):
    torch.manual_seed(0)
    B, C, H, W, Cout, k = 2, 8, 17, 19, 12, 3
    x = torch.randn(B, C, H, W, device=dev)
    w = torch.randn(Cout, C // cfg["groups"], k, k, device=dev) * 0.2
    bias = torch.randn(Cout, device=dev)
    Ho = (H + 2 * cfg["padding"] - (cfg["dilation"] * (k - 1) + 1)) // cfg["stride"] + 1
    Wo = (W + 2 * cfg["padding"] - (cfg["dilation"] * (k - 1) + 1)) // cfg["stride"] + 1
    off = torch.randn(B, cfg["dg"] * 2 * k * k, Ho, Wo, device=dev) * 2.0
    mask = torch.rand(B, cfg["dg"] * k * k, Ho, Wo, device=dev) if modulated else None
    args = (cfg["stride"], cfg["padding"], cfg["dilation"], cfg["groups"], cfg["dg"])
    leaves = [t.clone().requires_grad_() for t in (x, off, w, bias)] + \
        ([mask.clone().requires_grad_()] if modulated else [])
    ref_leaves = [t.detach().clone().requires_grad_() for t in leaves]
    y = deform_conv2d(leaves[0], leaves[1], leaves[2], leaves[3], leaves[4] if modulated else None, *args)
    yr = deform_conv2d_reference(ref_leaves[0], ref_leaves[1], ref_leaves[2], ref_leaves[3],
                                 ref_leaves[4] if modulated else None, *args)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for a, b, name in zip(leaves, ref_leaves, ["input", "offset", "weight", "bias", "mask"]):
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-3, atol=1e-3, msg=name)


def test_deform_conv_bf16_forward():
    torch.manual_seed(1)
    x = torch.randn(2, 16, 20, 20, device=dev)
    w = torch.randn(32, 16, 3, 3, device=dev) * 0.1
    off = torch.randn(2, 18, 20, 20, device=dev)
    y = deform_conv2d(x.bfloat16(), off, w.bfloat16(), None, None, 1, 1)
    yr = deform_conv2d_reference(x, off, w, None, None, 1, 1)
    assert y.dtype == torch.bfloat16
    torch.testing.assert_close(y.float(), yr, rtol=3e-2, atol=5e-2)


@pytest.mark.parametrize("no_trans", [True, False])
def test_deform_psroi_fwd_bwd(no_trans):
    torch.manual_seed(2)
    N, H, W, out_dim, gs, P, S = 2, 20, 24, 4, 3, 3, 3
    C = out_dim * gs * gs
    data = torch.randn(N, C, H, W, device=dev)
    # RoIs (and small part offsets) keep every sample inside the clamp range, where the
    # kernel's gradient (which, like the original, ignores the clamp) is exact
    rois = torch.tensor([[0, 4.0, 4.0, 30.0, 25.0], [1, 2.0, 2.0, 40.0, 30.0], [0, 10.0, 11.5, 14.0, 16.0],
                         [1, 20.0, 16.0, 36.0, 30.0]], device=dev)
    trans = None if no_trans else (torch.rand(4, 2, P, P, device=dev) * 0.2 - 0.1)
    d1 = data.clone().requires_grad_()
    d2 = data.clone().requires_grad_()
    t1 = None if no_trans else trans.clone().requires_grad_()
    t2 = None if no_trans else trans.clone().requires_grad_()
    y = deform_roi_pooling(d1, rois, t1, 0.5, P, out_dim, no_trans, gs, P, S, 0.2)
    yr = deform_roi_pooling_reference(d2, rois, t2, 0.5, P, out_dim, no_trans, gs, P, S, 0.2)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(d1.grad, d2.grad, rtol=1e-4, atol=1e-4)
    if not no_trans:
        torch.testing.assert_close(t1.grad, t2.grad, rtol=2e-3, atol=2e-3)


def test_psroi_rejects_bad_batch_index():
    data = torch.randn(1, 4, 8, 8, device=dev)
    rois = torch.tensor([[3, 0.0, 0.0, 4.0, 4.0]], device=dev)
    with pytest.raises(RuntimeError):
        deform_roi_pooling(data, rois, None, 1.0, 2, 1, True, 2, 2, 2, 0.0)
