"""Detection ops with HIP kernels (csrc/vision.hip) and torch references: nms, batched_nms,
roi_align, roi_pool, sigmoid_focal_loss -- the Mask R-CNN csrc entry points (reference
maskrcnn_benchmark/csrc/vision.cpp:11-24)."""
from __future__ import annotations

from typing import Tuple

import torch


def _native():
    from cloudtik_amd import ops
    return ops.require_native()


def _use_native(*ts) -> bool:
    from cloudtik_amd import ops
    return ops._use_native(*ts)


# ---------------------------------------------------------------------- NMS
def _box_iou(a, b, offset=0.0):
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt + offset).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    area = lambda x: (x[:, 2] - x[:, 0] + offset) * (x[:, 3] - x[:, 1] + offset)
    return inter / (area(a)[:, None] + area(b)[None, :] - inter).clamp(min=1e-12)


def nms_reference(boxes, scores, iou_threshold, offset=0.0):
    order = scores.argsort(descending=True)
    b = boxes[order].float()
    iou = _box_iou(b, b, offset)
    n = b.shape[0]
    removed = torch.zeros(n, dtype=torch.bool)
    keep = []
    iou_cpu = iou.cpu()
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        removed |= iou_cpu[i] > iou_threshold
    return order[torch.tensor(keep, dtype=torch.long, device=boxes.device)] if keep else order[:0]


def nms(boxes: torch.Tensor, scores: torch.Tensor, iou_threshold: float, offset: float = 0.0) -> torch.Tensor:
    """Indices of kept boxes, by decreasing score (torchvision.ops.nms semantics; ``offset=1``
    gives the legacy +1 box-area convention of maskrcnn_benchmark)."""
    if boxes.is_cuda and _use_native(boxes):
        order = scores.argsort(descending=True)
        keep = _native().nms_sorted(boxes[order].float().contiguous(), float(iou_threshold), float(offset))
        return order[keep]
    return nms_reference(boxes, scores, iou_threshold, offset)


def nms_segments(boxes: torch.Tensor, offsets, iou_threshold: float, offset: float = 0.0) -> torch.Tensor:
    """Keep mask (bool [N]) for many independent NMS problems at once: segment ``s`` is rows
    ``offsets[s]:offsets[s+1]`` of ``boxes``, each segment already sorted by decreasing score.
    On the GPU this is ONE mask launch + one reduction launch with a workgroup per segment
    (csrc/vision.hip ``nms_*_seg_kernel``), so the serial chunk walk is as long as the largest
    segment instead of the sum of all of them (the box-shift trick)."""
    off = torch.as_tensor(offsets, dtype=torch.long).cpu().contiguous()
    if boxes.is_cuda and _use_native(boxes):
        return _native().nms_segmented(boxes.float().contiguous(), off, float(iou_threshold), float(offset)).bool()
    keep = torch.zeros(boxes.shape[0], dtype=torch.bool, device=boxes.device)
    for s in range(off.numel() - 1):
        lo, hi = int(off[s]), int(off[s + 1])
        if hi > lo:
            b = boxes[lo:hi]
            # sorted already: the reference's argsort of a decreasing ramp is the identity
            k = nms_reference(b, torch.arange(hi - lo, 0, -1, device=b.device, dtype=torch.float32),
                              iou_threshold, offset)
            keep[lo + k] = True
    return keep


def batched_nms(boxes, scores, idxs, iou_threshold, offset=0.0):
    """NMS per category: boxes of different ``idxs`` never suppress each other.  Returns kept
    indices by decreasing score.  On the GPU every category is its own segment of one
    segmented-NMS launch (one host sync for the segment sizes)."""
    if boxes.numel() == 0:
        return torch.empty(0, dtype=torch.long, device=boxes.device)
    if boxes.is_cuda and _use_native(boxes):
        order = scores.argsort(descending=True, stable=True)
        order = order[idxs[order].argsort(stable=True)]             # (category, score desc)
        _, counts = torch.unique_consecutive(idxs[order], return_counts=True)
        off = torch.zeros(counts.numel() + 1, dtype=torch.long)
        off[1:] = counts.cpu().cumsum(0)
        kept = order[nms_segments(boxes[order], off, iou_threshold, offset)]
        return kept[scores[kept].argsort(descending=True, stable=True)]
    shift = idxs.to(boxes.dtype)[:, None] * (boxes.max() + 1 + offset)
    return nms(boxes + shift, scores, iou_threshold, offset)


# ---------------------------------------------------------------------- ROIAlign
def _bilinear_ref(f, y, x):
    C, H, W = f.shape
    valid = (y >= -1) & (y <= H) & (x >= -1) & (x <= W)
    y = y.clamp(min=0)
    x = x.clamp(min=0)
    y0 = y.floor().long()
    x0 = x.floor().long()
    ycap = y0 >= H - 1
    xcap = x0 >= W - 1
    y0 = torch.where(ycap, torch.full_like(y0, H - 1), y0)
    x0 = torch.where(xcap, torch.full_like(x0, W - 1), x0)
    y = torch.where(ycap, y0.float(), y)
    x = torch.where(xcap, x0.float(), x)
    y1 = torch.where(ycap, y0, y0 + 1)
    x1 = torch.where(xcap, x0, x0 + 1)
    ly, lx = y - y0, x - x0
    hy, hx = 1 - ly, 1 - lx
    v = (hy * hx) * f[:, y0, x0] + (hy * lx) * f[:, y0, x1] + (ly * hx) * f[:, y1, x0] + (ly * lx) * f[:, y1, x1]
    return v * valid


def roi_align_reference(feat, rois, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=False):
    PH, PW = output_size
    K = rois.shape[0]
    C = feat.shape[1]
    out = torch.zeros(K, C, PH, PW, dtype=torch.float32, device=feat.device)
    off = 0.5 if aligned else 0.0
    for k in range(K):
        b = int(rois[k, 0])
        x0, y0, x1, y1 = [float(v) * spatial_scale - off for v in rois[k, 1:]]
        rw, rh = x1 - x0, y1 - y0
        if not aligned:
            rw, rh = max(rw, 1.0), max(rh, 1.0)
        bw, bh = rw / PW, rh / PH
        gh = sampling_ratio if sampling_ratio > 0 else int(torch.tensor(rh / PH).ceil())
        gw = sampling_ratio if sampling_ratio > 0 else int(torch.tensor(rw / PW).ceil())
        f = feat[b].float()
        for ph in range(PH):
            for pw in range(PW):
                ys = torch.tensor([y0 + ph * bh + (iy + 0.5) * bh / gh for iy in range(gh)], device=feat.device)
                xs = torch.tensor([x0 + pw * bw + (ix + 0.5) * bw / gw for ix in range(gw)], device=feat.device)
                yy, xx = torch.meshgrid(ys, xs, indexing="ij")
                v = _bilinear_ref(f, yy.reshape(-1), xx.reshape(-1))
                out[k, :, ph, pw] = v.sum(-1) / max(gh * gw, 1)
    return out


class _RoiAlignFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, rois, output_size, scale, sr, aligned):
        ctx.save_for_backward(rois)
        ctx.meta = (list(feat.shape), scale, sr, aligned)
        return _native().roi_align_fwd(feat.contiguous(), rois.float().contiguous(), scale, output_size[0],
                                       output_size[1], sr, aligned)

    @staticmethod
    def backward(ctx, g):
        (rois,) = ctx.saved_tensors
        shape, scale, sr, aligned = ctx.meta
        return (_native().roi_align_bwd(g.contiguous(), rois.float().contiguous(), shape, scale, sr, aligned),
                None, None, None, None, None)


class _RoiAlignNHWCFn(torch.autograd.Function):
    """One launch over 1-5 NHWC pyramid levels; ``lvl`` (int32 [K] or None) is each RoI's
    level.  Backward returns every level's gradient from one shared zeroed fp32 buffer."""

    @staticmethod
    def forward(ctx, rois, lvl, output_size, scales, sr, aligned, *feats):
        rois = rois.float().contiguous()
        ctx.save_for_backward(rois, lvl)
        shapes = [d for f in feats for d in f.shape]
        ctx.meta = (shapes, list(scales), sr, aligned)
        return _native().roi_align_nhwc_fwd(list(feats), rois, lvl, list(scales), output_size[0], output_size[1],
                                            sr, aligned)

    @staticmethod
    def backward(ctx, g):
        rois, lvl = ctx.saved_tensors
        shapes, scales, sr, aligned = ctx.meta
        grads = _native().roi_align_nhwc_bwd(g, rois, lvl, shapes, scales, sr, aligned)
        return (None, None, None, None, None, None, *grads)


def _nhwc_ok(f: torch.Tensor) -> bool:
    return f.dim() == 4 and f.shape[1] % 8 == 0 and f.shape[1] > 1 and \
        f.is_contiguous(memory_format=torch.channels_last)


def roi_align_multilevel(feats, rois, levels, output_size, scales, sampling_ratio: int = 2, aligned: bool = False):
    """Pool every RoI from its own pyramid level: ``levels[k]`` indexes ``feats`` / ``scales``.

    On the GPU (channels_last maps) this is one kernel for all levels and all RoIs -- no
    per-level split, so no host sync; elsewhere a per-level loop over ``roi_align``."""
    if isinstance(output_size, int):
        output_size = (output_size, output_size)
    if feats[0].is_cuda and _use_native(feats[0]) and all(_nhwc_ok(f) for f in feats) and len(feats) <= 5:
        lvl = levels.to(torch.int32).contiguous() if len(feats) > 1 else None
        return _RoiAlignNHWCFn.apply(rois, lvl, tuple(output_size), tuple(float(s) for s in scales),
                                     int(sampling_ratio), bool(aligned), *feats)
    out = None
    for l, (f, s) in enumerate(zip(feats, scales)):
        idx = torch.nonzero(levels == l).squeeze(1)
        if idx.numel() == 0:
            continue
        o = roi_align(f, rois[idx], output_size, s, sampling_ratio, aligned)
        if out is None:
            out = o.new_zeros((rois.shape[0],) + tuple(o.shape[1:]))
            if o.is_contiguous(memory_format=torch.channels_last) and o.is_cuda:
                out = out.contiguous(memory_format=torch.channels_last)
        out = out.index_copy(0, idx, o.to(out.dtype))
    if out is None:
        out = feats[0].new_zeros(rois.shape[0], feats[0].shape[1], *output_size)
    return out


def roi_align_vectorized(feat, rois, output_size, spatial_scale=1.0, sampling_ratio=2, aligned=False):
    """Vectorised (autograd-differentiable) ROIAlign for a fixed ``sampling_ratio`` > 0: the
    CPU path of detection models (same sampling rule as ``roi_align_reference``)."""
    PH, PW = output_size
    K = rois.shape[0]
    N, C, H, W = feat.shape
    if K == 0:
        return feat.new_zeros(0, C, PH, PW)
    g = int(sampling_ratio)
    off = 0.5 if aligned else 0.0
    r = rois.float()
    b = r[:, 0].long()
    x0, y0 = r[:, 1] * spatial_scale - off, r[:, 2] * spatial_scale - off
    rw, rh = r[:, 3] * spatial_scale - off - x0, r[:, 4] * spatial_scale - off - y0
    if not aligned:
        rw, rh = rw.clamp(min=1.0), rh.clamp(min=1.0)
    frac_y = (torch.arange(PH * g, device=feat.device, dtype=torch.float32) + 0.5) / (PH * g)
    frac_x = (torch.arange(PW * g, device=feat.device, dtype=torch.float32) + 0.5) / (PW * g)
    ys = y0[:, None] + frac_y[None] * rh[:, None]            # [K, PH*g]
    xs = x0[:, None] + frac_x[None] * rw[:, None]            # [K, PW*g]
    yy = ys[:, :, None].expand(K, PH * g, PW * g)
    xx = xs[:, None, :].expand(K, PH * g, PW * g)
    valid = (yy >= -1) & (yy <= H) & (xx >= -1) & (xx <= W)
    yy, xx = yy.clamp(min=0), xx.clamp(min=0)
    y0i, x0i = yy.floor().long(), xx.floor().long()
    ycap, xcap = y0i >= H - 1, x0i >= W - 1
    y0i, x0i = torch.where(ycap, H - 1, y0i), torch.where(xcap, W - 1, x0i)
    yy, xx = torch.where(ycap, y0i.float(), yy), torch.where(xcap, x0i.float(), xx)
    y1i, x1i = torch.where(ycap, y0i, y0i + 1), torch.where(xcap, x0i, x0i + 1)
    ly, lx = yy - y0i, xx - x0i
    hy, hx = 1 - ly, 1 - lx
    f = feat.permute(0, 2, 3, 1).reshape(N * H * W, C).float()
    base = (b * H * W)[:, None, None]

    def tap(yi, xi):
        return f[(base + yi * W + xi).reshape(-1)].reshape(K, PH * g, PW * g, C)
    v = ((hy * hx)[..., None] * tap(y0i, x0i) + (hy * lx)[..., None] * tap(y0i, x1i)
         + (ly * hx)[..., None] * tap(y1i, x0i) + (ly * lx)[..., None] * tap(y1i, x1i))
    v = v * valid[..., None]
    v = v.reshape(K, PH, g, PW, g, C).mean(dim=(2, 4))
    return v.permute(0, 3, 1, 2).to(feat.dtype)


def roi_align(feat, rois, output_size, spatial_scale: float = 1.0, sampling_ratio: int = -1, aligned: bool = False):
    """feat [N, C, H, W]; rois [K, 5] = (batch_idx, x1, y1, x2, y2) -> [K, C, PH, PW]."""
    if isinstance(output_size, int):
        output_size = (output_size, output_size)
    if feat.is_cuda and _use_native(feat):
        if _nhwc_ok(feat):
            # NHWC maps (FPN pyramids): vectorised channel-contiguous kernel, channels_last output
            return _RoiAlignNHWCFn.apply(rois, None, tuple(output_size), (float(spatial_scale),),
                                         int(sampling_ratio), bool(aligned), feat)
        return _RoiAlignFn.apply(feat, rois, tuple(output_size), float(spatial_scale), int(sampling_ratio), bool(aligned))
    if sampling_ratio > 0:
        return roi_align_vectorized(feat, rois, output_size, spatial_scale, sampling_ratio, aligned)
    return roi_align_reference(feat, rois, output_size, spatial_scale, sampling_ratio, aligned).to(feat.dtype)


# ---------------------------------------------------------------------- ROIPool
def roi_pool_reference(feat, rois, output_size, spatial_scale=1.0):
    PH, PW = output_size
    K, C, H, W = rois.shape[0], feat.shape[1], feat.shape[2], feat.shape[3]
    out = torch.zeros(K, C, PH, PW, dtype=torch.float32, device=feat.device)
    for k in range(K):
        b = int(rois[k, 0])
        x0, y0, x1, y1 = [int(round(float(v) * spatial_scale)) for v in rois[k, 1:]]
        rw, rh = max(x1 - x0 + 1, 1), max(y1 - y0 + 1, 1)
        bw, bh = rw / PW, rh / PH
        import math
        for ph in range(PH):
            hs = min(max(int(math.floor(ph * bh)) + y0, 0), H)
            he = min(max(int(math.ceil((ph + 1) * bh)) + y0, 0), H)
            for pw in range(PW):
                ws = min(max(int(math.floor(pw * bw)) + x0, 0), W)
                we = min(max(int(math.ceil((pw + 1) * bw)) + x0, 0), W)
                if he > hs and we > ws:
                    out[k, :, ph, pw] = feat[b, :, hs:he, ws:we].float().amax(dim=(-1, -2))
    return out


class _RoiPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feat, rois, output_size, scale):
        out, arg = _native().roi_pool_fwd(feat.contiguous(), rois.float().contiguous(), scale, output_size[0],
                                          output_size[1])
        ctx.save_for_backward(rois, arg)
        ctx.shape = list(feat.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        rois, arg = ctx.saved_tensors
        return _native().roi_pool_bwd(g.contiguous(), rois.float().contiguous(), arg, ctx.shape), None, None, None


def roi_pool(feat, rois, output_size, spatial_scale: float = 1.0):
    if isinstance(output_size, int):
        output_size = (output_size, output_size)
    if feat.is_cuda and _use_native(feat):
        return _RoiPoolFn.apply(feat, rois, tuple(output_size), float(spatial_scale))
    return roi_pool_reference(feat, rois, output_size, spatial_scale).to(feat.dtype)


# ---------------------------------------------------------------------- SigmoidFocalLoss
def sigmoid_focal_loss_reference(logits, targets, gamma, alpha):
    N, C = logits.shape
    x = logits.float()
    cls = torch.arange(1, C + 1, device=logits.device)[None, :]
    t = targets[:, None]
    c1 = (t == cls).float()
    c2 = ((t >= 0) & (t != cls)).float()
    p = torch.sigmoid(x)
    term1 = (1 - p) ** gamma * torch.log(p.clamp(min=torch.finfo(torch.float32).tiny))
    term2 = p ** gamma * torch.nn.functional.logsigmoid(-x)
    return -c1 * alpha * term1 - c2 * (1 - alpha) * term2


class _FocalFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, targets, gamma, alpha):
        logits, targets = logits.contiguous(), targets.contiguous()
        ctx.save_for_backward(logits, targets)
        ctx.gamma, ctx.alpha = gamma, alpha
        return _native().focal_fwd(logits, targets, gamma, alpha)

    @staticmethod
    def backward(ctx, g):
        logits, targets = ctx.saved_tensors
        return _native().focal_bwd(logits, targets, g.float().contiguous(), ctx.gamma, ctx.alpha), None, None, None


def sigmoid_focal_loss(logits, targets, gamma: float = 2.0, alpha: float = 0.25, reduction: str = "sum"):
    """maskrcnn_benchmark semantics: targets in 1..C are foreground classes, 0 background,
    negative entries ignored.  Returns per-element losses reduced by ``reduction``."""
    if logits.is_cuda and _use_native(logits):
        loss = _FocalFn.apply(logits, targets.to(torch.int64), float(gamma), float(alpha))
    else:
        loss = sigmoid_focal_loss_reference(logits, targets, gamma, alpha)
    if reduction == "sum":
        return loss.sum()
    if reduction == "mean":
        return loss.mean()
    return loss


# ---------------------------------------------------------------------- image ingest
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def images_to_tensor_reference(images: torch.Tensor, flip=None, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    x = images.float() / 255.0
    if flip is not None:
        x = torch.where(flip.bool()[:, None, None, None], x.flip(2), x)
    x = (x - torch.tensor(mean, device=x.device)) / torch.tensor(std, device=x.device)
    return x.permute(0, 3, 1, 2)


def images_to_tensor(images: torch.Tensor, flip: torch.Tensor = None, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """uint8 [N, H, W, 3] -> normalised [N, 3, H, W] (bf16 channels_last on the GPU, one HIP
    pass with optional per-image horizontal flip; fp32 on the CPU)."""
    if images.is_cuda and _use_native(images):
        f = None if flip is None else flip.to(torch.uint8).contiguous()
        return _native().image_u8_to_bf16(images.contiguous(), f, list(map(float, mean)), list(map(float, std)))
    return images_to_tensor_reference(images, flip, mean, std)
