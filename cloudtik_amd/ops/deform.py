"""Deformable convolution v1/v2 and deformable PS RoI pooling (reference
maskrcnn_benchmark/layers/dcn/deform_conv_func.py:9-260, deform_conv_module.py:10-190,
deform_pool_func.py:8-100, deform_pool_module.py:6-170).

GPU: bilinear sampling kernels from csrc/deform.hip + per-group GEMMs (hipBLASLt).  CPU:
a ``grid_sample`` formulation with identical zero-padding semantics; autograd through it is
also the fp32 reference the GPU tests compare the hand-written backward against.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


def _native():
    from cloudtik_amd import ops
    return ops.require_native()


def _use_native(*ts) -> bool:
    from cloudtik_amd import ops
    return ops._use_native(*ts)


def _pair(v) -> Tuple[int, int]:
    return (v, v) if isinstance(v, int) else tuple(v)


# ---------------------------------------------------------------------- reference
def _sample_positions(B, H, W, Ho, Wo, kh, kw, stride, padding, dilation, offset, dg, device):
    """[B, dg, K, Ho, Wo] sampling rows / cols."""
    K = kh * kw
    ho = torch.arange(Ho, device=device, dtype=torch.float32) * stride[0] - padding[0]
    wo = torch.arange(Wo, device=device, dtype=torch.float32) * stride[1] - padding[1]
    ki = torch.arange(kh, device=device, dtype=torch.float32).repeat_interleave(kw) * dilation[0]
    kj = torch.arange(kw, device=device, dtype=torch.float32).repeat(kh) * dilation[1]
    off = offset.view(B, dg, K, 2, Ho, Wo).float()
    h = ho.view(1, 1, 1, Ho, 1) + ki.view(1, 1, K, 1, 1) + off[:, :, :, 0]
    w = wo.view(1, 1, 1, 1, Wo) + kj.view(1, 1, K, 1, 1) + off[:, :, :, 1]
    return h, w


def deform_conv2d_reference(input, offset, weight, bias=None, mask=None, stride=1, padding=0, dilation=1,
                            groups=1, deformable_groups=1):
    stride, padding, dilation = _pair(stride), _pair(padding), _pair(dilation)
    B, C, H, W = input.shape
    Cout, Cg, kh, kw = weight.shape
    K = kh * kw
    Ho = (H + 2 * padding[0] - (dilation[0] * (kh - 1) + 1)) // stride[0] + 1
    Wo = (W + 2 * padding[1] - (dilation[1] * (kw - 1) + 1)) // stride[1] + 1
    dg = deformable_groups
    h, w = _sample_positions(B, H, W, Ho, Wo, kh, kw, stride, padding, dilation, offset, dg, input.device)
    # grid_sample(align_corners=True): pixel centre i <-> -1 + 2 i / (size - 1)
    gy = 2 * h / max(H - 1, 1) - 1
    gx = 2 * w / max(W - 1, 1) - 1
    grid = torch.stack([gx, gy], dim=-1).view(B * dg, K * Ho, Wo, 2)
    x = input.float().view(B * dg, C // dg, H, W)
    s = F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True)
    s = s.view(B, dg, C // dg, K, Ho, Wo)
    if mask is not None:
        s = s * mask.float().view(B, dg, 1, K, Ho, Wo)
    cols = s.reshape(B, C, K, Ho * Wo).reshape(B, groups, (C // groups) * K, Ho * Wo)
    wg = weight.float().view(groups, Cout // groups, Cg * K)
    out = torch.einsum("gok,bgkn->bgon", wg, cols).reshape(B, Cout, Ho, Wo)
    if bias is not None:
        out = out + bias.float().view(1, -1, 1, 1)
    return out.to(input.dtype)


# ---------------------------------------------------------------------- HIP path
class _DeformConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, offset, mask, weight, bias, stride, padding, dilation, groups, dg):
        C = _native()
        B, Cin, H, W = input.shape
        Cout, Cg, kh, kw = weight.shape
        input = input.contiguous()
        offset = offset.float().contiguous()
        mask = None if mask is None else mask.float().contiguous()
        geo = ([kh, kw], list(stride), list(padding), list(dilation), dg)
        cols = C.dcn_im2col(input, offset, mask, *geo)                      # [Cin*K, B*Ho*Wo]
        Ho = (H + 2 * padding[0] - (dilation[0] * (kh - 1) + 1)) // stride[0] + 1
        Wo = (W + 2 * padding[1] - (dilation[1] * (kw - 1) + 1)) // stride[1] + 1
        K = kh * kw
        wg = weight.view(groups, Cout // groups, Cg * K).to(cols.dtype)
        out = torch.bmm(wg, cols.view(groups, Cg * K, B * Ho * Wo))          # [g, Cout/g, B*Ho*Wo]
        out = out.view(Cout, B, Ho, Wo).permute(1, 0, 2, 3)
        if bias is not None:
            out = out + bias.to(out.dtype).view(1, -1, 1, 1)
        ctx.save_for_backward(input, offset, mask, weight, cols)
        ctx.geo, ctx.groups, ctx.has_bias = geo, groups, bias is not None
        ctx.shape = (B, Ho, Wo)
        return out.contiguous()

    @staticmethod
    def backward(ctx, gout):
        C = _native()
        input, offset, mask, weight, cols = ctx.saved_tensors
        B, Ho, Wo = ctx.shape
        g = ctx.groups
        Cout, Cg, kh, kw = weight.shape
        K = kh * kw
        go = gout.float().permute(1, 0, 2, 3).reshape(g, Cout // g, B * Ho * Wo)
        wg = weight.float().view(g, Cout // g, Cg * K)
        gcol = torch.bmm(wg.transpose(1, 2), go).reshape(g * Cg * K, B * Ho * Wo).contiguous()
        gin = C.dcn_col2im(gcol, input, offset, mask, *ctx.geo).to(input.dtype)
        goff, gmask = C.dcn_col2coord(gcol, input, offset, mask, *ctx.geo)
        gw = torch.bmm(go, cols.float().view(g, Cg * K, B * Ho * Wo).transpose(1, 2)).view_as(weight).to(weight.dtype)
        gb = gout.float().sum((0, 2, 3)).to(weight.dtype) if ctx.has_bias else None
        return gin, goff, (gmask if mask is not None else None), gw, gb, None, None, None, None, None


def deform_conv2d(input, offset, weight, bias=None, mask=None, stride=1, padding=0, dilation=1, groups=1,
                  deformable_groups=1):
    """Deformable convolution; ``mask`` given -> modulated (DCNv2)."""
    stride, padding, dilation = _pair(stride), _pair(padding), _pair(dilation)
    if input.is_cuda and _use_native(input):
        return _DeformConvFn.apply(input, offset, mask, weight, bias, stride, padding, dilation, groups,
                                   deformable_groups)
    return deform_conv2d_reference(input, offset, weight, bias, mask, stride, padding, dilation, groups,
                                   deformable_groups)


class DeformConv(nn.Module):
    """DCNv1 layer: forward(input, offset)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 deformable_groups=1, bias=False):
        super().__init__()
        assert in_channels % groups == 0 and out_channels % groups == 0
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride, self.padding, self.dilation = _pair(stride), _pair(padding), _pair(dilation)
        self.groups, self.deformable_groups = groups, deformable_groups
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels // groups, *self.kernel_size))
        self.bias = nn.Parameter(torch.zeros(out_channels)) if bias else None
        n = in_channels * self.kernel_size[0] * self.kernel_size[1]
        nn.init.uniform_(self.weight, -1.0 / math.sqrt(n), 1.0 / math.sqrt(n))

    def _offset_channels(self, per=2):
        return self.deformable_groups * per * self.kernel_size[0] * self.kernel_size[1]

    def forward(self, input, offset, mask=None):
        return deform_conv2d(input, offset, self.weight, self.bias, mask, self.stride, self.padding, self.dilation,
                             self.groups, self.deformable_groups)


class ModulatedDeformConv(DeformConv):
    """DCNv2 layer: forward(input, offset, mask)."""

    def __init__(self, *a, bias=True, **kw):
        super().__init__(*a, bias=bias, **kw)


class ModulatedDeformConvPack(ModulatedDeformConv):
    """DCNv2 with its own offset/mask predictor (zero-initialised: starts as a plain conv)."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.conv_offset_mask = nn.Conv2d(self.in_channels, self._offset_channels(3), self.kernel_size,
                                          self.stride, self.padding, self.dilation, bias=True)
        nn.init.zeros_(self.conv_offset_mask.weight)
        nn.init.zeros_(self.conv_offset_mask.bias)

    def forward(self, input):
        out = self.conv_offset_mask(input)
        o1, o2, m = torch.chunk(out, 3, dim=1)
        return super().forward(input, torch.cat([o1, o2], 1), torch.sigmoid(m))


# ---------------------------------------------------------------------- deformable PS RoI pooling
def deform_roi_pooling_reference(data, rois, offset, spatial_scale, out_size, out_channels, no_trans,
                                 group_size=1, part_size=None, sample_per_part=4, trans_std=0.0):
    part = out_size if part_size is None else part_size
    N, C, H, W = data.shape
    Kr = rois.shape[0]
    dev = data.device
    P, S = out_size, sample_per_part
    r = rois.float()
    rnd = lambda v: torch.sign(v) * torch.floor(v.abs() + 0.5)     # C round(): half away from zero
    x1 = rnd(r[:, 1]) * spatial_scale - 0.5
    y1 = rnd(r[:, 2]) * spatial_scale - 0.5
    x2 = (rnd(r[:, 3]) + 1) * spatial_scale - 0.5
    y2 = (rnd(r[:, 4]) + 1) * spatial_scale - 0.5
    rw = (x2 - x1).clamp(min=0.1)
    rh = (y2 - y1).clamp(min=0.1)
    bw, bh = rw / P, rh / P
    p = torch.arange(P, device=dev)
    part_idx = torch.floor(p.float() / P * part).long()
    ctop = torch.arange(out_channels, device=dev)
    if no_trans or offset is None or offset.numel() == 0:
        tx = torch.zeros(Kr, out_channels, P, P, device=dev)
        ty = torch.zeros_like(tx)
    else:
        nc = offset.shape[1] // 2
        cls = ctop // (out_channels // nc)
        t = offset.float().view(Kr, nc, 2, part, part)[:, :, :, part_idx][:, :, :, :, part_idx]   # [Kr,nc,2,P,P]
        tx = t[:, cls, 0] * trans_std
        ty = t[:, cls, 1] * trans_std
    wstart = p.view(1, 1, 1, P) * bw.view(-1, 1, 1, 1) + x1.view(-1, 1, 1, 1) + tx * rw.view(-1, 1, 1, 1)
    hstart = p.view(1, 1, P, 1) * bh.view(-1, 1, 1, 1) + y1.view(-1, 1, 1, 1) + ty * rh.view(-1, 1, 1, 1)
    s = torch.arange(S, device=dev, dtype=torch.float32)
    w = wstart[..., None, None] + s.view(1, 1, 1, 1, 1, S) * (bw / S).view(-1, 1, 1, 1, 1, 1)
    h = hstart[..., None, None] + s.view(1, 1, 1, 1, S, 1) * (bh / S).view(-1, 1, 1, 1, 1, 1)
    w, h = torch.broadcast_tensors(w, h)                                      # [Kr, Co, P, P, S, S]
    valid = (w >= -0.5) & (w <= W - 0.5) & (h >= -0.5) & (h <= H - 0.5)
    w = w.clamp(0, W - 1)
    h = h.clamp(0, H - 1)
    g = torch.clamp(torch.floor(p.float() * group_size / P).long(), 0, group_size - 1)
    cin = (ctop.view(-1, 1, 1) * group_size + g.view(1, -1, 1)) * group_size + g.view(1, 1, -1)   # [Co, P(h), P(w)]
    b = r[:, 0].long()
    x0, y0 = torch.floor(w).long(), torch.floor(h).long()
    xc, yc = torch.ceil(w).long(), torch.ceil(h).long()
    dx, dy = w - x0, h - y0
    base = data.reshape(N, C, H * W)
    bi = b.view(-1, 1, 1, 1, 1, 1).expand_as(x0)
    ci = cin.view(1, out_channels, P, P, 1, 1).expand_as(x0)

    def at(yy, xx):
        return base[bi, ci, yy * W + xx]
    val = (1 - dx) * (1 - dy) * at(y0, x0) + (1 - dx) * dy * at(yc, x0) + dx * (1 - dy) * at(y0, xc) + dx * dy * at(yc, xc)
    val = torch.where(valid, val, torch.zeros_like(val))
    cnt = valid.sum((-1, -2)).float()
    out = val.sum((-1, -2)) / cnt.clamp(min=1)
    return torch.where(cnt > 0, out, torch.zeros_like(out))


class _DeformPsroiFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, rois, offset, spatial_scale, out_size, out_channels, no_trans, group_size, part_size,
                sample_per_part, trans_std):
        trans = None if (no_trans or offset is None or offset.numel() == 0) else offset.float().contiguous()
        args = (float(spatial_scale), int(out_channels), int(group_size), int(out_size), int(part_size),
                int(sample_per_part), float(trans_std))
        out, cnt = _native().psroi_fwd(data.contiguous(), rois.float().contiguous(), trans, *args)
        ctx.save_for_backward(data, rois, trans if trans is not None else torch.empty(0, device=data.device), cnt)
        ctx.args, ctx.has_trans = args, trans is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        data, rois, trans, cnt = ctx.saved_tensors
        gdata, gtrans = _native().psroi_bwd(gout.contiguous().float(), data.contiguous(), rois.float().contiguous(),
                                            trans if ctx.has_trans else None, cnt, *ctx.args)
        return gdata, None, (gtrans if ctx.has_trans else None), None, None, None, None, None, None, None, None


def deform_roi_pooling(data, rois, offset, spatial_scale, out_size, out_channels, no_trans, group_size=1,
                       part_size=None, sample_per_part=4, trans_std=0.0):
    part = out_size if part_size is None else part_size
    if not 0.0 <= trans_std <= 1.0:
        raise ValueError("trans_std must be in [0, 1]")
    if data.is_cuda and _use_native(data):
        return _DeformPsroiFn.apply(data.float(), rois, offset, spatial_scale, out_size, out_channels, no_trans,
                                    group_size, part, sample_per_part, trans_std)
    return deform_roi_pooling_reference(data, rois, offset, spatial_scale, out_size, out_channels, no_trans,
                                        group_size, part, sample_per_part, trans_std)


class DeformRoIPooling(nn.Module):
    def __init__(self, spatial_scale, out_size, out_channels, no_trans, group_size=1, part_size=None,
                 sample_per_part=4, trans_std=0.0):
        super().__init__()
        self.spatial_scale, self.out_size, self.out_channels = spatial_scale, out_size, out_channels
        self.no_trans, self.group_size = no_trans, group_size
        self.part_size = out_size if part_size is None else part_size
        self.sample_per_part, self.trans_std = sample_per_part, trans_std

    def forward(self, data, rois, offset=None):
        return deform_roi_pooling(data, rois, None if self.no_trans else offset, self.spatial_scale, self.out_size,
                                  self.out_channels, self.no_trans, self.group_size, self.part_size,
                                  self.sample_per_part, self.trans_std)


class DeformRoIPoolingPack(DeformRoIPooling):
    """Predicts the part offsets from a first, offset-free pooling pass (fc head, zero-init)."""

    def __init__(self, *a, deform_fc_channels=1024, **kw):
        super().__init__(*a, **kw)
        if not self.no_trans:
            d = self.out_size * self.out_size * self.out_channels
            self.offset_fc = nn.Sequential(nn.Linear(d, deform_fc_channels), nn.ReLU(inplace=True),
                                           nn.Linear(deform_fc_channels, deform_fc_channels), nn.ReLU(inplace=True),
                                           nn.Linear(deform_fc_channels, self.out_size * self.out_size * 2))
            nn.init.zeros_(self.offset_fc[-1].weight)
            nn.init.zeros_(self.offset_fc[-1].bias)

    def forward(self, data, rois):
        if self.no_trans:
            return super().forward(data, rois)
        n = rois.shape[0]
        x = deform_roi_pooling(data, rois, None, self.spatial_scale, self.out_size, self.out_channels, True,
                               self.group_size, self.part_size, self.sample_per_part, self.trans_std)
        offset = self.offset_fc(x.view(n, -1)).view(n, 2, self.out_size, self.out_size)
        return deform_roi_pooling(data, rois, offset, self.spatial_scale, self.out_size, self.out_channels, False,
                                  self.group_size, self.part_size, self.sample_per_part, self.trans_std)
