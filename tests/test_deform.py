"""Deformable conv / deformable PS RoI pooling references on CPU, checked against a direct
per-sample loop of the DCN definition (zero-padded bilinear sampling)."""
import math

import numpy as np
import torch

from cloudtik_amd.ops.deform import (DeformRoIPoolingPack, ModulatedDeformConvPack, deform_conv2d_reference,
                                     deform_roi_pooling_reference)


def _bilinear(im, h, w):
    H, W = im.shape
    if h <= -1 or w <= -1 or h >= H or w >= W:
        return 0.0
    h0, w0 = math.floor(h), math.floor(w)
    lh, lw = h - h0, w - w0
    v = 0.0
    for (y, x, wt) in ((h0, w0, (1 - lh) * (1 - lw)), (h0, w0 + 1, (1 - lh) * lw),
                       (h0 + 1, w0, lh * (1 - lw)), (h0 + 1, w0 + 1, lh * lw)):
        if 0 <= y < H and 0 <= x < W:
            v += wt * im[y, x]
    return v


def test_deform_conv_reference_matches_loop():
    torch.manual_seed(0)
    B, C, H, W, Cout, k, dg, groups = 2, 4, 6, 7, 6, 3, 2, 2
    x = torch.randn(B, C, H, W, dtype=torch.float64)
    w = torch.randn(Cout, C // groups, k, k, dtype=torch.float64)
    bias = torch.randn(Cout, dtype=torch.float64)
    stride, pad, dil = 1, 1, 1
    Ho, Wo = H, W
    off = torch.randn(B, dg * 2 * k * k, Ho, Wo, dtype=torch.float64) * 1.5
    mask = torch.rand(B, dg * k * k, Ho, Wo, dtype=torch.float64)
    got = deform_conv2d_reference(x.float(), off.float(), w.float(), bias.float(), mask.float(), stride, pad, dil,
                                  groups, dg).double()
    xn, on, mn, wn = x.numpy(), off.numpy(), mask.numpy(), w.numpy()
    want = np.zeros((B, Cout, Ho, Wo))
    cpg_in, cpg_out = C // groups, Cout // groups
    for b in range(B):
        for o in range(Cout):
            gi = o // cpg_out
            for ho in range(Ho):
                for wo in range(Wo):
                    acc = bias[o].item()
                    for ci in range(cpg_in):
                        c = gi * cpg_in + ci
                        g = c // (C // dg)
                        for i in range(k):
                            for j in range(k):
                                p = i * k + j
                                h = ho * stride - pad + i * dil + on[b, g * 2 * k * k + 2 * p, ho, wo]
                                ww = wo * stride - pad + j * dil + on[b, g * 2 * k * k + 2 * p + 1, ho, wo]
                                acc += wn[o, ci, i, j] * mn[b, g * k * k + p, ho, wo] * _bilinear(xn[b, c], h, ww)
                    want[b, o, ho, wo] = acc
    np.testing.assert_allclose(got.numpy(), want, rtol=1e-4, atol=1e-4)


def test_zero_offset_dcn_equals_conv():
    torch.manual_seed(1)
    m = ModulatedDeformConvPack(8, 16, 3, padding=1, stride=2)
    x = torch.randn(2, 8, 9, 11)
    # zero-initialised offsets, sigmoid(0) = 0.5 mask
    want = torch.nn.functional.conv2d(x, m.weight * 0.5, m.bias, stride=2, padding=1)
    torch.testing.assert_close(m(x), want, rtol=1e-4, atol=1e-5)


def test_psroi_reference_loop_and_pack():
    torch.manual_seed(2)
    N, H, W, out_dim, gs, P, S = 2, 12, 14, 3, 2, 3, 2
    C = out_dim * gs * gs
    data = torch.randn(N, C, H, W)
    rois = torch.tensor([[0, 1.0, 2.0, 9.0, 8.0], [1, 0.0, 0.0, 13.0, 11.0], [0, 5.0, 5.5, 6.0, 7.0]])
    trans = torch.randn(3, 2, P, P) * 0.3
    got = deform_roi_pooling_reference(data, rois, trans, 0.5, P, out_dim, False, gs, P, S, 0.1)
    want = torch.zeros_like(got)
    rnd = lambda v: math.floor(abs(v) + 0.5) * (1 if v >= 0 else -1)
    for n in range(3):
        b = int(rois[n, 0])
        x1, y1 = rnd(float(rois[n, 1])) * 0.5 - 0.5, rnd(float(rois[n, 2])) * 0.5 - 0.5
        x2, y2 = (rnd(float(rois[n, 3])) + 1) * 0.5 - 0.5, (rnd(float(rois[n, 4])) + 1) * 0.5 - 0.5
        rw, rh = max(x2 - x1, 0.1), max(y2 - y1, 0.1)
        for c in range(out_dim):
            for ph in range(P):
                for pw in range(P):
                    tx = float(trans[n, 0, ph, pw]) * 0.1
                    ty = float(trans[n, 1, ph, pw]) * 0.1
                    ws = pw * rw / P + x1 + tx * rw
                    hs = ph * rh / P + y1 + ty * rh
                    gw, gh = min(pw * gs // P, gs - 1), min(ph * gs // P, gs - 1)
                    cin = (c * gs + gh) * gs + gw
                    tot, cnt = 0.0, 0
                    for ih in range(S):
                        for iw in range(S):
                            w = ws + iw * rw / P / S
                            h = hs + ih * rh / P / S
                            if w < -0.5 or w > W - 0.5 or h < -0.5 or h > H - 0.5:
                                continue
                            w, h = min(max(w, 0), W - 1), min(max(h, 0), H - 1)
                            tot += _bilinear(data[b, cin].double().numpy(), h, w)
                            cnt += 1
                    want[n, c, ph, pw] = tot / cnt if cnt else 0.0
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)
    pack = DeformRoIPoolingPack(0.5, P, out_dim, False, group_size=gs, sample_per_part=S, trans_std=0.1,
                                deform_fc_channels=32)
    assert pack(data, rois).shape == (3, out_dim, P, P)
