"""Box and mask heads of Faster / Mask R-CNN (reference: maskrcnn_benchmark
``modeling/roi_heads/{box_head,mask_head}/*`` and ``modeling/poolers.py``, SURVEY.md §2.12 /
native components N3-N4).

* ``MultiScaleRoIAlign`` assigns each RoI to a pyramid level (``k = 4 + log2(sqrt(area)/224)``,
  clamped to the available levels) and pools it with the HIP ROIAlign kernel
  (``ops.roi_align_multilevel``, bwd by atomics into the feature maps); ONE launch for all
  levels -- the kernel reads each RoI's level, so there is no per-level split and no host sync.
* Mask targets are produced by the same ROIAlign kernel: the ground-truth masks are treated
  as a batch of one-channel images and every positive proposal is pooled from the mask of
  its matched object (``rois[:, 0]`` = gt index) to 28x28 -- no CPU polygon rasterisation.
* Inference: softmax, class-specific decode, score threshold, per-class HIP NMS
  (``ops.batched_nms``), top detections per image; masks are the sigmoid of the predicted
  class channel on the kept boxes.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd import ops
from cloudtik_amd.models.detection import box_ops as B


def _pad_rows(x: torch.Tensor, rows: int) -> torch.Tensor:
    """Zero-pad dim 0 up to ``rows`` (the step's upper bound).  The mask head's batch is the
    number of RoIs, which changes every step; MIOpen selects (and may compile) a convolution
    solution per problem shape, so padding to the fixed bound keeps ONE warm shape."""
    n = x.shape[0]
    k = max(rows, n)
    if k == n:
        return x
    pad = x.new_zeros((k - n,) + tuple(x.shape[1:]))
    out = torch.cat([x, pad], 0)
    return out.contiguous(memory_format=torch.channels_last) if x.is_contiguous(
        memory_format=torch.channels_last) and x.dim() == 4 else out


def _to_rois(boxes: List[torch.Tensor]) -> torch.Tensor:
    return torch.cat([torch.cat([torch.full((b.shape[0], 1), float(i), device=b.device, dtype=torch.float32),
                                 b.float()], 1) for i, b in enumerate(boxes)], 0)


class MultiScaleRoIAlign(nn.Module):
    def __init__(self, strides: Sequence[int], output_size: int, sampling_ratio: int = 2,
                 canonical_scale: float = 224.0, canonical_level: int = 4, aligned: bool = False):
        super().__init__()
        self.strides = list(strides)
        self.output_size = output_size
        self.sampling_ratio = sampling_ratio
        self.aligned = aligned
        self.k_min = int(round(math.log2(self.strides[0])))
        self.k_max = int(round(math.log2(self.strides[-1])))
        self.canonical_scale, self.canonical_level = canonical_scale, canonical_level

    def level_of(self, rois: torch.Tensor) -> torch.Tensor:
        s = torch.sqrt(B.box_area(rois[:, 1:]))
        k = torch.floor(self.canonical_level + torch.log2(s / self.canonical_scale + 1e-6))
        return (k.clamp(self.k_min, self.k_max) - self.k_min).long()

    def forward(self, feats: List[torch.Tensor], boxes: List[torch.Tensor]) -> torch.Tensor:
        rois = _to_rois(boxes)
        feats = feats[:len(self.strides)]
        if len(feats) == 1:
            return ops.roi_align(feats[0], rois, self.output_size, 1.0 / self.strides[0], self.sampling_ratio,
                                 self.aligned)
        return ops.roi_align_multilevel(feats, rois, self.level_of(rois), self.output_size,
                                        [1.0 / s for s in self.strides], self.sampling_ratio, self.aligned)


class TwoMLPHead(nn.Module):
    def __init__(self, in_features: int, hidden: int = 1024, device=None, dtype=None):
        super().__init__()
        self.fc6 = nn.Linear(in_features, hidden, device=device, dtype=dtype)
        self.fc7 = nn.Linear(hidden, hidden, device=device, dtype=dtype)

    def forward(self, x):
        return F.relu(self.fc7(F.relu(self.fc6(x.flatten(1)))))


class BoxPredictor(nn.Module):
    def __init__(self, hidden: int, num_classes: int, device=None, dtype=None):
        super().__init__()
        self.cls_score = nn.Linear(hidden, num_classes, device=device, dtype=dtype)
        self.bbox_pred = nn.Linear(hidden, num_classes * 4, device=device, dtype=dtype)
        nn.init.normal_(self.cls_score.weight, std=0.01)
        nn.init.normal_(self.bbox_pred.weight, std=0.001)
        nn.init.zeros_(self.cls_score.bias)
        nn.init.zeros_(self.bbox_pred.bias)

    def forward(self, x):
        return self.cls_score(x), self.bbox_pred(x)


class MaskHead(nn.Module):
    """4 x (3x3 conv + ReLU) -> 2x2 stride-2 deconv + ReLU -> per-class 1x1 projection.

    The 1x1 projection is evaluated as a matrix product on the NHWC activations.  With
    ``labels`` (training targets / predicted classes) only the one class each RoI needs is
    computed -- a batched GEMV [K, 784, 256] x [K, 256] instead of all 81 class maps
    (1/81 of the FLOPs and no 81-channel convolution, whose channel count fits no MFMA tile).
    """

    def __init__(self, channels: int, num_classes: int, layers: int = 4, dim: int = 256, device=None, dtype=None):
        super().__init__()
        convs, c = [], channels
        for _ in range(layers):
            conv = nn.Conv2d(c, dim, 3, 1, 1, device=device, dtype=torch.float32)
            nn.init.kaiming_normal_(conv.weight, mode="fan_out", nonlinearity="relu")
            nn.init.zeros_(conv.bias)
            convs.append(conv)
            c = dim
        self.convs = nn.ModuleList(convs)
        self.deconv = nn.ConvTranspose2d(dim, dim, 2, 2, device=device, dtype=torch.float32)
        self.logits = nn.Linear(dim, num_classes, device=device, dtype=torch.float32)
        nn.init.kaiming_normal_(self.deconv.weight, mode="fan_out", nonlinearity="relu")
        nn.init.normal_(self.logits.weight, std=0.001)
        nn.init.zeros_(self.deconv.bias)
        nn.init.zeros_(self.logits.bias)
        if dtype is not None:
            self.to(dtype)

    def forward(self, x, labels: Optional[torch.Tensor] = None):
        for c in self.convs:
            x = F.relu(c(x))
        h = F.relu(self.deconv(x))
        K, D, H, W = h.shape
        hp = h.permute(0, 2, 3, 1).reshape(K, H * W, D)            # free view for NHWC
        if labels is None:
            return F.linear(hp, self.logits.weight, self.logits.bias).reshape(K, H, W, -1).permute(0, 3, 1, 2)
        w = self.logits.weight[labels]                                # [K, D]
        out = torch.bmm(hp, w.unsqueeze(-1)).squeeze(-1) + self.logits.bias[labels].unsqueeze(-1)
        return out.reshape(K, H, W)


class RoIHeads(nn.Module):
    def __init__(self, channels: int, strides: Sequence[int], num_classes: int, with_mask: bool = True,
                 box_pool: int = 7, mask_pool: int = 14, hidden: int = 1024, fg_iou: float = 0.5,
                 bg_iou: float = 0.5, batch_size_per_image: int = 512, positive_fraction: float = 0.25,
                 score_thresh: float = 0.05, nms_thresh: float = 0.5, detections_per_img: int = 100,
                 device=None, dtype=None):
        super().__init__()
        roi_strides = [s for s in strides if s <= 32]
        self.box_pool = MultiScaleRoIAlign(roi_strides, box_pool, 2)
        self.box_head = TwoMLPHead(channels * box_pool * box_pool, hidden, device, dtype)
        self.box_predictor = BoxPredictor(hidden, num_classes, device, dtype)
        self.with_mask = with_mask
        if with_mask:
            self.mask_pool = MultiScaleRoIAlign(roi_strides, mask_pool, 2)
            self.mask_head = MaskHead(channels, num_classes, device=device, dtype=dtype)
        self.num_classes = num_classes
        self.matcher = B.Matcher(fg_iou, bg_iou, allow_low_quality=False)
        self.coder = B.BoxCoder((10.0, 10.0, 5.0, 5.0))
        self.batch_size_per_image, self.positive_fraction = batch_size_per_image, positive_fraction
        self.score_thresh, self.nms_thresh, self.detections_per_img = score_thresh, nms_thresh, detections_per_img
        self.pad_mask_rois = device is not None and torch.device(device).type == "cuda"

    # ------------------------------------------------------------------ training
    def _sample(self, proposals, targets):
        """Fixed-size, sync-free RoI sampling: every image yields exactly
        ``batch_size_per_image`` rows (fewer only if it has fewer candidates), ordered
        positives first, then negatives, then padding rows (label -1, ignored by the losses).
        Sampling is the batched top-k draw of ``B.sample_pos_neg_batched``, so no step waits
        for a nonzero() on the host, and the box / mask heads always see the same shapes."""
        S = self.batch_size_per_image
        cands, labs, mids = [], [], []
        for p, t in zip(proposals, targets):
            gt = t["boxes"].to(p)
            p = torch.cat([p, gt])                     # ground truth joins the proposals
            if gt.numel():
                m = self.matcher(B.box_iou(gt, p))
                lab = t["labels"].to(p.device)[m.clamp(min=0)].long()
                lab = torch.where(m == B.Matcher.BELOW_LOW, 0, torch.where(m == B.Matcher.BETWEEN, -1, lab))
            else:
                m = torch.full((p.shape[0],), -1, device=p.device, dtype=torch.long)
                lab = torch.zeros_like(m)
            cands.append(p)
            labs.append(lab)
            mids.append(m.clamp(min=0))
        L = max(c.shape[0] for c in cands)
        pad = lambda xs, v: torch.stack([F.pad(x, (0, 0) * (x.dim() - 1) + (0, L - x.shape[0]), value=v)  # noqa: E731
                                         for x in xs])
        cand, lab, mid = pad(cands, 0.0), pad(labs, -1), pad(mids, 0)
        # padding candidates become 1x1 boxes (never sampled: label -1), so pooling and box
        # encoding stay finite
        n_real = torch.tensor([c.shape[0] for c in cands], device=cand.device)
        is_pad = torch.arange(L, device=cand.device)[None, :] >= n_real[:, None]
        cand = torch.where(is_pad[..., None], cand.new_tensor([0.0, 0.0, 1.0, 1.0]), cand)
        pm, nm = B.sample_pos_neg_batched(lab, S, self.positive_fraction)
        key = torch.where(pm, 0, torch.where(nm, 1, 2))
        order = key.sort(dim=1, stable=True).indices[:, :min(S, L)]
        valid = key.gather(1, order) < 2
        sel_p = cand.gather(1, order[..., None].expand(-1, -1, 4))
        sel_lab = torch.where(valid, lab.gather(1, order), -1)
        sel_m = mid.gather(1, order)
        tgts = []
        for n, t in enumerate(targets):
            gt = t["boxes"].to(sel_p)
            tgts.append(self.coder.encode(gt[sel_m[n]], sel_p[n]) if gt.numel() else torch.zeros_like(sel_p[n]))
        return list(sel_p.unbind(0)), sel_lab, torch.stack(tgts), sel_m

    def forward(self, feats: List[torch.Tensor], proposals: List[torch.Tensor], image_sizes: List[Tuple[int, int]],
                targets: Optional[List[Dict[str, torch.Tensor]]] = None):
        if self.training and targets is not None:
            props, labels, reg_t, gt_idx = self._sample(proposals, targets)
        else:
            props = proposals
        x = self.box_head(self.box_pool(feats, props))
        cls, reg = self.box_predictor(x)
        cls, reg = cls.float(), reg.float()
        if self.training and targets is not None:
            lab = labels.reshape(-1)
            tgt = reg_t.reshape(-1, 4)
            n_valid = (lab >= 0).sum().clamp(min=1)
            loss_cls = F.cross_entropy(cls, lab, ignore_index=-1, reduction="sum") / n_valid
            pos = (lab > 0).float()
            r = reg.view(reg.shape[0], -1, 4).gather(1, lab.clamp(min=0)[:, None, None].expand(-1, 1, 4))[:, 0]
            # non-positive rows (negatives, padding, zero-width proposals whose encoded targets
            # are inf) regress onto themselves: zero loss AND zero, finite gradient
            tgt = torch.where(pos[:, None] > 0, tgt, r.detach())
            loss_box = B.smooth_l1(r, tgt, beta=1.0 / 9, reduction="none").sum() / n_valid
            losses = {"loss_classifier": loss_cls, "loss_box_reg": loss_box}
            if self.with_mask:
                losses["loss_mask"] = self._mask_loss(feats, props, labels, gt_idx, targets)
            return None, losses
        return self._postprocess(feats, cls, reg, props, image_sizes), {}

    def _mask_loss(self, feats, props, labels, gt_idx, targets):
        """Positives sit in the first ``P`` rows of every image (``_sample``'s order), so the
        mask head always runs on exactly N x P RoIs; non-positive rows carry zero weight."""
        P = min(int(self.batch_size_per_image * self.positive_fraction), labels.shape[1])
        M = self.mask_head_size
        boxes = [p[:P] for p in props]
        lab = labels[:, :P]
        w = (lab > 0).float()
        tgts = []
        for p, gi, t in zip(boxes, gt_idx[:, :P], targets):
            masks = t["masks"]
            if masks.shape[0] == 0:
                tgts.append(torch.zeros(P, M, M, device=p.device))
                continue
            masks = masks.to(device=p.device, dtype=torch.float32)[:, None]            # [G, 1, H, W]
            rois = torch.cat([gi.float()[:, None], p.float()], 1)
            tgts.append((ops.roi_align(masks, rois, M, 1.0, 2, True)[:, 0] >= 0.5).float())
        x = self.mask_pool(feats, boxes)
        logits = self.mask_head(x, lab.clamp(min=0).reshape(-1)).float()
        bce = F.binary_cross_entropy_with_logits(logits, torch.cat(tgts), reduction="none").mean((1, 2))
        return (bce * w.reshape(-1)).sum() / w.sum().clamp(min=1)

    def _mask_rows(self, bound: int) -> int:
        return bound if self.pad_mask_rois else 0

    @property
    def mask_head_size(self) -> int:
        return self.mask_pool.output_size * 2

    # ------------------------------------------------------------------ inference
    @torch.no_grad()
    def _postprocess(self, feats, cls, reg, props, image_sizes):
        counts = [p.shape[0] for p in props]
        probs = F.softmax(cls, -1).split(counts)
        boxes = self.coder.decode(reg, torch.cat(props)).split(counts)
        K = self.num_classes
        results = []
        for pr, bx, size in zip(probs, boxes, image_sizes):
            bx = B.clip_boxes(bx.reshape(-1, 4), size).reshape(-1, K, 4)[:, 1:].reshape(-1, 4)
            sc = pr[:, 1:].reshape(-1)
            lab = torch.arange(1, K, device=sc.device).repeat(pr.shape[0])
            keep = torch.nonzero(sc > self.score_thresh).squeeze(1)
            bx, sc, lab = bx[keep], sc[keep], lab[keep]
            keep = B.remove_small(bx, 1e-2)
            bx, sc, lab = bx[keep], sc[keep], lab[keep]
            keep = ops.batched_nms(bx, sc, lab, self.nms_thresh)[:self.detections_per_img]
            results.append({"boxes": bx[keep], "scores": sc[keep], "labels": lab[keep]})
        if self.with_mask:
            dets = [r["boxes"] for r in results]
            n = sum(d.shape[0] for d in dets)
            if n:
                lab = torch.cat([r["labels"] for r in results])
                bound = self._mask_rows(self.detections_per_img * len(dets))
                x = _pad_rows(self.mask_pool(feats, dets), bound)
                m = torch.sigmoid(self.mask_head(x, _pad_rows(lab, bound))[:n].float())
                for r, mm in zip(results, m.split([d.shape[0] for d in dets])):
                    r["masks"] = mm[:, None]
            else:
                for r in results:
                    r["masks"] = torch.zeros(0, 1, self.mask_head_size, self.mask_head_size, device=cls.device)
        return results


def paste_masks(masks: torch.Tensor, boxes: torch.Tensor, size: Tuple[int, int], threshold: float = 0.5) -> torch.Tensor:
    """[D, 1, M, M] mask probabilities in box coordinates -> [D, H, W] boolean image masks
    (one ``grid_sample`` for all detections)."""
    D = masks.shape[0]
    H, W = size
    if D == 0:
        return torch.zeros(0, H, W, dtype=torch.bool, device=masks.device)
    ys = torch.arange(H, device=masks.device, dtype=torch.float32) + 0.5
    xs = torch.arange(W, device=masks.device, dtype=torch.float32) + 0.5
    x1, y1, x2, y2 = [boxes[:, i:i + 1].float() for i in range(4)]
    gx = (xs[None] - x1) / (x2 - x1).clamp(min=1e-3) * 2 - 1           # [D, W]
    gy = (ys[None] - y1) / (y2 - y1).clamp(min=1e-3) * 2 - 1           # [D, H]
    grid = torch.stack([gx[:, None, :].expand(D, H, W), gy[:, :, None].expand(D, H, W)], -1)
    img = F.grid_sample(masks.float(), grid, align_corners=False, padding_mode="zeros")
    return img[:, 0] >= threshold
