"""Detection model family (Mask R-CNN, Faster R-CNN, RetinaNet, SSD-ResNet34,
SSD-MobileNet, YOLOv4, ResNeXt): box utilities against brute-force references, tiny-config
train/eval steps on CPU, and bf16 steps through the HIP NMS / ROIAlign / focal-loss kernels
on the GPU."""
import math

import pytest
import torch

from cloudtik_amd.models.detection import box_ops as B
from cloudtik_amd.models.detection import GeneralizedRCNN, synthetic_detection_batch


def test_box_coder_roundtrip_and_iou():
    g = torch.Generator().manual_seed(0)
    ref = torch.rand(50, 2, generator=g) * 100
    ref = torch.cat([ref, ref + 5 + torch.rand(50, 2, generator=g) * 50], 1)
    gt = torch.rand(50, 2, generator=g) * 100
    gt = torch.cat([gt, gt + 5 + torch.rand(50, 2, generator=g) * 50], 1)
    for w in ((1, 1, 1, 1), (10, 10, 5, 5)):
        c = B.BoxCoder(w)
        torch.testing.assert_close(c.decode(c.encode(gt, ref), ref), gt, atol=1e-3, rtol=1e-4)
    iou = B.box_iou(gt[:7], ref[:9])
    for i in range(7):
        for j in range(9):
            a, b = gt[i].tolist(), ref[j].tolist()
            iw = max(0, min(a[2], b[2]) - max(a[0], b[0]))
            ih = max(0, min(a[3], b[3]) - max(a[1], b[1]))
            inter = iw * ih
            u = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
            assert abs(iou[i, j].item() - inter / u) < 1e-5


def test_matcher_thresholds_and_low_quality():
    iou = torch.tensor([[0.9, 0.45, 0.2, 0.1], [0.1, 0.3, 0.35, 0.05]])
    m = B.Matcher(0.7, 0.3)(iou)
    assert m.tolist() == [0, B.Matcher.BETWEEN, B.Matcher.BETWEEN, B.Matcher.BELOW_LOW]
    m = B.Matcher(0.7, 0.3, allow_low_quality=True)(iou)
    assert m.tolist() == [0, B.Matcher.BETWEEN, 1, B.Matcher.BELOW_LOW]


def test_anchor_generator_counts_and_centres():
    ag = B.AnchorGenerator([[32], [64]], (0.5, 1.0, 2.0), strides=(4, 8))
    feats = [torch.zeros(1, 1, 10, 12), torch.zeros(1, 1, 5, 6)]
    a = ag(feats)
    assert a[0].shape == (10 * 12 * 3, 4) and a[1].shape == (5 * 6 * 3, 4)
    cx = (a[1][:, 0] + a[1][:, 2]) / 2
    assert torch.allclose(cx[:3], torch.zeros(3)) and torch.allclose(cx[3:6], torch.full((3,), 8.0))
    area = B.box_area(a[0][:3])
    assert torch.allclose(area, torch.full((3,), 32.0 ** 2), rtol=1e-5)


def test_vectorized_roi_align_matches_loop_reference():
    from cloudtik_amd.ops.vision import roi_align_reference, roi_align_vectorized
    g = torch.Generator().manual_seed(3)
    f = torch.randn(2, 6, 15, 11, generator=g)
    r = torch.tensor([[0, 1., 2, 9, 11], [1, -3, -2, 20, 15], [0, 4.2, 5.1, 4.9, 6.3], [1, 10, 8, 16.9, 12.9]])
    for aligned in (False, True):
        torch.testing.assert_close(roi_align_vectorized(f, r, (7, 5), 0.5, 2, aligned),
                                   roi_align_reference(f, r, (7, 5), 0.5, 2, aligned), atol=1e-5, rtol=1e-5)


def _tiny_rcnn(with_mask=True, **kw):
    return GeneralizedRCNN(num_classes=5, depth=18, fpn_channels=32, representation=64, rpn_pre_nms=(200, 100),
                           rpn_post_nms=(100, 50), box_batch_per_image=64, with_mask=with_mask, **kw)


def test_mask_rcnn_train_and_eval_cpu():
    torch.manual_seed(0)
    m = _tiny_rcnn(dtype=torch.float32)
    imgs, tg = synthetic_detection_batch(2, 128, 5, 4)
    losses = m(imgs, tg)
    assert set(losses) == {"loss_objectness", "loss_rpn_box_reg", "loss_classifier", "loss_box_reg", "loss_mask"}
    total = sum(losses.values())
    assert torch.isfinite(total)
    total.backward()
    assert m.roi_heads.mask_head.logits.weight.grad.abs().sum() > 0
    assert m.rpn.head.cls.weight.grad.abs().sum() > 0
    assert m.backbone.body.conv1.weight.grad is None          # frozen stem
    m.eval()
    with torch.no_grad():
        dets = m(imgs)
    for d in dets:
        n = d["boxes"].shape[0]
        assert d["scores"].shape == (n,) and d["labels"].shape == (n,) and d["masks"].shape == (n, 1, 28, 28)
        assert (d["labels"] >= 1).all() and (d["labels"] < 5).all()


def test_mask_rcnn_learns_fixed_batch_cpu():
    """A few SGD steps on one batch must lower the detector's total loss."""
    torch.manual_seed(0)
    m = _tiny_rcnn(with_mask=False, dtype=torch.float32)
    imgs, tg = synthetic_detection_batch(2, 128, 5, 3, with_masks=False)
    opt = torch.optim.SGD([p for p in m.parameters() if p.requires_grad], lr=0.02, momentum=0.9)
    first = None
    for _ in range(12):
        torch.manual_seed(1)                                   # same proposal sampling each step
        loss = sum(m(imgs, tg).values())
        first = first if first is not None else float(loss)
        opt.zero_grad()
        loss.backward()
        opt.step()
    assert float(loss) < first


def test_paste_masks():
    from cloudtik_amd.models.detection import paste_masks
    masks = torch.ones(1, 1, 28, 28)
    img = paste_masks(masks, torch.tensor([[10., 20., 30., 60.]]), (80, 50))
    ys, xs = torch.nonzero(img[0], as_tuple=True)
    assert ys.min() == 20 and ys.max() == 59 and xs.min() == 10 and xs.max() == 29


def test_retinanet_cpu():
    from cloudtik_amd.models.detection.retinanet import RetinaNet
    torch.manual_seed(0)
    m = RetinaNet(num_classes=4, depth=18, fpn_channels=32, dtype=torch.float32)
    imgs, tg = synthetic_detection_batch(2, 128, 5, 4, with_masks=False)
    l = m(imgs, tg)
    sum(l.values()).backward()
    assert all(torch.isfinite(v) for v in l.values())
    m.eval()
    m.score_thresh = 0.0
    with torch.no_grad():
        d = m(imgs)
    assert d[0]["boxes"].shape[0] == 100 and (d[0]["labels"] >= 1).all() and (d[0]["labels"] <= 4).all()


def test_ssd_default_boxes_and_training_cpu():
    from cloudtik_amd.models.detection.ssd import (ssd300_default_boxes, ssd300_mobilenet_v1,
                                                    ssd_mobilenet_default_boxes)
    assert len(ssd300_default_boxes()) == 8732
    assert len(ssd_mobilenet_default_boxes()) == 1917
    torch.manual_seed(0)
    m = ssd300_mobilenet_v1(num_classes=5, dtype=torch.float32)
    imgs, tg = synthetic_detection_batch(2, 300, 5, 4, with_masks=False)
    l = m(imgs, tg)["loss"]
    assert torch.isfinite(l)
    l.backward()
    # matching: every object gets at least its best default box
    labels, _ = m.match(tg, 300)
    assert all(int((labels[i] > 0).sum()) >= tg[i]["boxes"].shape[0] for i in range(2))
    m.eval()
    with torch.no_grad():
        loc, conf = m(imgs)
    assert loc.shape == (2, 1917, 4) and conf.shape == (2, 1917, 5)
    r = m.postprocess(loc, conf, 300)
    assert r[0]["boxes"].shape[1] == 4


def test_ssd_resnet34_param_count():
    from cloudtik_amd.models.detection.ssd import ssd300_resnet34
    m = ssd300_resnet34(81, dtype=torch.float32)
    # ResNet-34 trunk (layers 1-3) + extras + heads of the MLPerf SSD
    assert 19e6 < sum(p.numel() for p in m.parameters()) < 25e6


def test_yolov4_shapes_cpu():
    from cloudtik_amd.models.detection.yolo import yolov4
    m = yolov4(num_classes=3, width=0.25, depth=(1, 1, 1, 1, 1), dtype=torch.float32).eval()
    with torch.no_grad():
        o = m(torch.randn(1, 3, 128, 128))
    assert [t.shape[-1] for t in o] == [16, 8, 4] and all(t.shape[1] == 3 * 8 for t in o)
    d = m.decode(o)
    assert d.shape == (1, 3 * (16 * 16 + 8 * 8 + 4 * 4), 8)
    r = m.postprocess(o, (128, 128), conf_thresh=0.05, max_candidates=500)
    assert r[0]["boxes"].shape[0] <= 300


def test_resnet_family_param_counts():
    from cloudtik_amd.models import resnet as R
    counts = {f: sum(p.numel() for p in getattr(R, f)(dtype=torch.float32).parameters())
              for f in ("resnet34", "resnext50_32x4d", "resnet101")}
    assert counts == {"resnet34": 21797672, "resnext50_32x4d": 25028904, "resnet101": 44549160}


# --------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_mask_rcnn_bf16_gpu(cuda):
    torch.manual_seed(0)
    m = _tiny_rcnn(device=cuda, dtype=torch.bfloat16)
    imgs, tg = synthetic_detection_batch(2, 256, 5, 4, device=cuda)
    losses = m(imgs, tg)
    total = sum(losses.values())
    assert torch.isfinite(total), losses
    total.backward()
    assert torch.isfinite(m.roi_heads.box_predictor.cls_score.weight.grad.float()).all()
    m.eval()
    with torch.no_grad():
        dets = m(imgs)
    assert dets[0]["masks"].shape[1:] == (1, 28, 28)


@pytest.mark.gpu
def test_detection_inference_gpu_matches_cpu_postprocess(cuda):
    """RetinaNet eval on GPU (HIP NMS) vs the same head outputs post-processed on CPU."""
    from cloudtik_amd.models.detection.retinanet import RetinaNet
    torch.manual_seed(0)
    m = RetinaNet(num_classes=4, depth=18, fpn_channels=32, device=cuda, dtype=torch.float32).eval()
    x = torch.randn(1, 3, 128, 128, device=cuda)
    with torch.no_grad():
        feats = m.backbone(x)
        cls, reg = m.head(feats)
        anchors = m.anchors(feats)
        g = m.postprocess(cls, reg, anchors, [(128, 128)])[0]
        c = m.postprocess([t.cpu() for t in cls], [t.cpu() for t in reg], [a.cpu() for a in anchors],
                          [(128, 128)])[0]
    torch.testing.assert_close(g["scores"].cpu(), c["scores"], atol=1e-5, rtol=1e-5)
    assert torch.equal(g["labels"].cpu(), c["labels"])


@pytest.mark.gpu
def test_retinanet_focal_ssd_yolo_gpu(cuda):
    from cloudtik_amd.models.detection.retinanet import RetinaNet
    from cloudtik_amd.models.detection.ssd import ssd300_resnet34
    from cloudtik_amd.models.detection.yolo import yolov4
    torch.manual_seed(0)
    m = RetinaNet(num_classes=4, depth=18, fpn_channels=32, device=cuda, dtype=torch.bfloat16)
    imgs, tg = synthetic_detection_batch(2, 256, 5, 4, with_masks=False, device=cuda)
    l = m(imgs, tg)
    sum(l.values()).backward()
    assert all(torch.isfinite(v) for v in l.values())
    s = ssd300_resnet34(5, device=cuda)
    imgs, tg = synthetic_detection_batch(2, 300, 5, 4, with_masks=False, device=cuda)
    ls = s(imgs, tg)["loss"]
    ls.backward()
    assert torch.isfinite(ls)
    y = yolov4(num_classes=80, device=cuda).eval()
    with torch.no_grad():
        o = y(torch.randn(2, 3, 416, 416, device=cuda))
        r = y.postprocess(o, (416, 416))
    assert len(r) == 2 and o[0].shape == (2, 255, 52, 52)


@pytest.mark.gpu
def test_frozen_bn_autograd_matches_reference(cuda):
    from cloudtik_amd import ops
    torch.manual_seed(0)
    C = 64
    x = torch.randn(4, C, 9, 11, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x)
    w, b = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda)
    rm, rv = torch.randn(C, device=cuda), torch.rand(C, device=cuda) + 0.5
    x1, r1 = x.clone().requires_grad_(), r.clone().requires_grad_()
    y = ops.batch_norm_act(x1, w, b, rm, rv, residual=r1, relu=True, training=False)
    g = torch.randn_like(y)
    y.backward(g)
    x2, r2 = x.float().clone().requires_grad_(), r.float().clone().requires_grad_()
    y2 = torch.relu(torch.nn.functional.batch_norm(x2, rm, rv, w, b, False, 0.1, 1e-5) + r2)
    y2.backward(g.float())
    torch.testing.assert_close(y.float(), y2, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(x1.grad.float(), x2.grad, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(r1.grad.float(), r2.grad, atol=3e-2, rtol=2e-2)


@pytest.mark.gpu
def test_nms_large_matches_reference(cuda):
    """5000 clustered boxes (many suppressions across chunks) vs the CPU greedy reference."""
    from cloudtik_amd import ops
    from cloudtik_amd.ops.vision import nms_reference
    g = torch.Generator().manual_seed(5)
    ctr = torch.rand(300, 2, generator=g) * 600
    pts = ctr[torch.randint(0, 300, (5000,), generator=g)] + torch.randn(5000, 2, generator=g) * 6
    wh = torch.rand(5000, 2, generator=g) * 40 + 10
    boxes = torch.cat([pts, pts + wh], 1)
    scores = torch.rand(5000, generator=g)
    keep = ops.nms(boxes.to(cuda), scores.to(cuda), 0.5).cpu()
    ref = nms_reference(boxes, scores, 0.5)
    # greedy-NMS invariants (robust to IoU rounding at exactly the threshold):
    # kept boxes are score-ordered and mutually below the threshold, and every dropped box
    # overlaps a higher-scored kept box
    eps = 1e-4
    assert (scores[keep][1:] <= scores[keep][:-1]).all()
    iou = B.box_iou(boxes[keep], boxes[keep]).triu(1)
    assert iou.max() <= 0.5 + eps
    dropped = torch.ones(5000, dtype=torch.bool)
    dropped[keep] = False
    d = torch.nonzero(dropped).squeeze(1)
    cover = (B.box_iou(boxes[keep], boxes[d]) > 0.5 - eps) & (scores[keep][:, None] > scores[d][None, :])
    assert cover.any(0).all()
    assert abs(keep.numel() - ref.numel()) <= 2


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("sr", [2, 3])
def test_roi_align_nhwc_matches_reference(cuda, dtype, sr):
    from cloudtik_amd import ops
    from cloudtik_amd.ops.vision import roi_align_vectorized
    g = torch.Generator().manual_seed(11)
    f = torch.randn(2, 64, 23, 31, generator=g)
    xy = torch.rand(40, 2, generator=g) * 25 - 2
    wh = torch.rand(40, 2, generator=g) * 30 + 0.5
    rois = torch.cat([torch.randint(0, 2, (40, 1), generator=g).float(), xy, xy + wh], 1)
    fg = f.to(cuda, dtype).contiguous(memory_format=torch.channels_last).requires_grad_()
    out = ops.roi_align(fg, rois.to(cuda), 7, 0.5, sr, True)
    assert out.is_contiguous(memory_format=torch.channels_last)
    fr = f.clone().requires_grad_()
    ref = roi_align_vectorized(fr, rois, (7, 7), 0.5, sr, True)
    tol = dict(atol=2e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(out.float().cpu(), ref.to(dtype).float(), **tol)
    go = torch.randn(ref.shape, generator=g)
    out.backward(go.to(cuda, dtype))
    ref.backward(go)
    torch.testing.assert_close(fg.grad.float().cpu(), fr.grad, **(dict(atol=5e-2, rtol=5e-2)
                                                                   if dtype == torch.bfloat16 else tol))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_roi_align_multilevel_matches_per_level(cuda, dtype):
    """One launch over 4 NHWC levels (each RoI reads its own level) vs the CPU per-level loop,
    forward and the per-level feature gradients."""
    from cloudtik_amd import ops
    g = torch.Generator().manual_seed(13)
    shapes = [(2, 32, 40, 48), (2, 32, 20, 24), (2, 32, 10, 12), (2, 32, 5, 6)]
    feats = [torch.randn(s, generator=g) for s in shapes]
    K = 60
    xy = torch.rand(K, 2, generator=g) * 150
    wh = torch.rand(K, 2, generator=g) * 120 + 2
    rois = torch.cat([torch.randint(0, 2, (K, 1), generator=g).float(), xy, xy + wh], 1)
    lvl = torch.randint(0, 4, (K,), generator=g)
    scales = [1 / 4, 1 / 8, 1 / 16, 1 / 32]
    fg = [f.to(cuda, dtype).contiguous(memory_format=torch.channels_last).requires_grad_() for f in feats]
    out = ops.roi_align_multilevel(fg, rois.to(cuda), lvl.to(cuda), 7, scales, 2, False)
    fr = [f.clone().requires_grad_() for f in feats]
    ref = ops.roi_align_multilevel(fr, rois, lvl, 7, scales, 2, False)
    tol = dict(atol=2e-2, rtol=2e-2) if dtype == torch.bfloat16 else dict(atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(out.float().cpu(), ref.to(dtype).float(), **tol)
    go = torch.randn(ref.shape, generator=g)
    out.backward(go.to(cuda, dtype))
    ref.backward(go)
    for a, b in zip(fg, fr):
        assert a.grad.shape == b.grad.shape
        torch.testing.assert_close(a.grad.float().cpu(), b.grad, **(dict(atol=5e-2, rtol=5e-2)
                                                                   if dtype == torch.bfloat16 else tol))


def test_sample_pos_neg_batched_counts_and_uniformity():
    g = torch.Generator().manual_seed(2)
    lab = torch.full((3, 1000), -1)
    lab[0, :50] = 1                     # few positives: all taken, negatives fill the rest
    lab[0, 50:900] = 0
    lab[1, :400] = 2                    # many positives: capped at 64
    lab[1, 400:] = 0
    lab[2, :10] = 0                     # almost nothing to draw from
    pm, nm = B.sample_pos_neg_batched(lab, 256, 0.25, generator=g)
    assert pm[0].sum() == 50 and nm[0].sum() == 206
    assert pm[1].sum() == 64 and nm[1].sum() == 192
    assert pm[2].sum() == 0 and nm[2].sum() == 10
    assert not (pm & nm).any() and (lab[pm] >= 1).all() and (lab[nm] == 0).all()
    hits = torch.zeros(400)
    for _ in range(200):
        p, _ = B.sample_pos_neg_batched(lab[1:2], 256, 0.25, generator=g)
        hits += p[0, :400].float()
    assert hits.min() > 0 and hits.max() < 4 * hits.mean()   # every positive gets drawn


def _clustered_boxes(n, seed, spread=600):
    g = torch.Generator().manual_seed(seed)
    ctr = torch.rand(max(n // 16, 1), 2, generator=g) * spread
    pts = ctr[torch.randint(0, ctr.shape[0], (n,), generator=g)] + torch.randn(n, 2, generator=g) * 6
    wh = torch.rand(n, 2, generator=g) * 40 + 10
    return torch.cat([pts, pts + wh], 1), torch.rand(n, generator=g)


def test_rpn_batched_selection_matches_per_image_cpu():
    """The all-images segmented-NMS proposal path keeps exactly what the per-image
    (level-shifted batched_nms) path keeps."""
    from cloudtik_amd.models.detection.rpn import RPN
    torch.manual_seed(0)
    ag = B.AnchorGenerator(((32,), (64,)), (0.5, 1.0, 2.0), (8, 16))
    rpn = RPN(16, ag, pre_nms_top_n=(300, 200), post_nms_top_n=(150, 100), min_size=2.0).eval()
    feats = [torch.randn(2, 16, 20, 24), torch.randn(2, 16, 10, 12)]
    sizes = [(150, 180), (160, 190)]
    with torch.no_grad():
        logits, deltas = rpn.head(feats)
        anchors = ag(feats)
        obj = [B.permute_flatten(l, 1).squeeze(-1).float() for l in logits]
        reg = [B.permute_flatten(d, 4).float() * 2 for d in deltas]
        got = rpn._select_batched(obj, reg, anchors, sizes)
        for n in range(2):
            dec = [rpn.coder.decode(r[n], a) for r, a in zip(reg, anchors)]
            ref = rpn._select([o[n] for o in obj], dec, sizes[n])
            assert got[n].shape == ref.shape
            torch.testing.assert_close(got[n], ref)


def test_nms_segments_cpu_matches_per_segment():
    from cloudtik_amd import ops
    from cloudtik_amd.ops.vision import nms_reference
    boxes, scores = _clustered_boxes(400, 3, spread=200)
    off = [0, 0, 130, 131, 400]
    sb, ss = [], []
    for lo, hi in zip(off[:-1], off[1:]):
        o = scores[lo:hi].argsort(descending=True)
        sb.append(boxes[lo:hi][o])
        ss.append(scores[lo:hi][o])
    b, s = torch.cat(sb), torch.cat(ss)
    keep = ops.nms_segments(b, off, 0.5)
    for lo, hi in zip(off[:-1], off[1:]):
        ref = torch.zeros(hi - lo, dtype=torch.bool)
        if hi > lo:
            ref[nms_reference(b[lo:hi], s[lo:hi], 0.5)] = True
        assert torch.equal(keep[lo:hi], ref)


@pytest.mark.gpu
def test_segmented_nms_gpu_matches_reference(cuda):
    """Segmented kernel: empty, single-box and multi-chunk segments in one launch, and
    batched_nms (category segments) vs the box-shift CPU path."""
    from cloudtik_amd import ops
    from cloudtik_amd.ops.vision import nms_reference
    boxes, scores = _clustered_boxes(3000, 7, spread=300)
    off = [0, 0, 1, 700, 700, 2999, 3000]
    b = torch.cat([boxes[lo:hi][scores[lo:hi].argsort(descending=True)] for lo, hi in zip(off[:-1], off[1:])])
    keep = ops.nms_segments(b.to(cuda), off, 0.6).cpu()
    ramp = torch.arange(3000, 0, -1).float()
    for lo, hi in zip(off[:-1], off[1:]):
        ref = torch.zeros(hi - lo, dtype=torch.bool)
        if hi > lo:
            ref[nms_reference(b[lo:hi], ramp[lo:hi], 0.6)] = True
        # ties at exactly the threshold may flip a box or two between fp paths
        assert (keep[lo:hi] != ref).sum() <= 2
    idx = torch.randint(0, 17, (3000,), generator=torch.Generator().manual_seed(1))
    got = ops.batched_nms(boxes.to(cuda), scores.to(cuda), idx.to(cuda), 0.5).cpu()
    ref = ops.batched_nms(boxes, scores, idx, 0.5)
    assert (scores[got][1:] <= scores[got][:-1]).all()
    assert len(set(got.tolist()) ^ set(ref.tolist())) <= 4
