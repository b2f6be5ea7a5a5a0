"""COCO data path (data/coco.py) and the Mask R-CNN training entry (examples/ai/maskrcnn_train.py):
RLE (both encodings) and polygon masks, box-AP evaluator, loader geometry, CPU train + eval."""
import importlib.util
import math
import os

import numpy as np
import pytest
import torch

from cloudtik_amd.data import coco as C

HERE = os.path.dirname(os.path.abspath(__file__))


def _rle_counts(mask):
    flat = mask.T.reshape(-1)                     # column-major
    counts, cur, run = [], 0, 0
    for v in flat:
        if v != cur:
            counts.append(run)
            cur, run = v, 0
        run += 1
    counts.append(run)
    return counts


def _rle_string(counts):                          # the compressed encoder, for the round trip
    out = []
    for i, x in enumerate(counts):
        if i > 2:
            x -= counts[i - 2]
        more = True
        while more:
            c = x & 0x1F
            x >>= 5
            more = (x != -1) if (c & 0x10) else (x != 0)
            if more:
                c |= 0x20
            out.append(chr(c + 48))
    return "".join(out)


def test_rle_decode_both_encodings():
    rng = np.random.default_rng(0)
    m = (rng.random((23, 31)) < 0.3).astype(np.uint8)
    m[5:15, 7:20] = 1
    counts = _rle_counts(m)
    assert np.array_equal(C.rle_decode({"counts": counts, "size": [23, 31]}, 23, 31), m)
    assert np.array_equal(C.rle_decode({"counts": _rle_string(counts), "size": [23, 31]}, 23, 31), m)


def test_polygon_mask_fills_rectangle():
    m = C.polygons_to_mask([[2, 3, 10, 3, 10, 8, 2, 8]], 12, 14)
    assert m[3:9, 2:11].all() and m.sum() == 6 * 9


def test_evaluate_bbox():
    gts = {1: {"boxes": np.array([[0, 0, 10, 10], [20, 20, 40, 40]], float), "labels": np.array([1, 2])},
           2: {"boxes": np.array([[5, 5, 25, 25]], float), "labels": np.array([1])}}
    perfect = {k: {"boxes": v["boxes"], "labels": v["labels"], "scores": np.ones(len(v["labels"]))}
               for k, v in gts.items()}
    assert C.evaluate_bbox(perfect, gts)["AP"] == pytest.approx(1.0)
    assert C.evaluate_bbox({}, gts)["AP"] == 0.0
    # a confident false positive ranked above the true positives lowers AP but not AP50 to 0
    noisy = {k: dict(v) for k, v in perfect.items()}
    noisy[1] = {"boxes": np.array([[100, 100, 120, 120], [0, 0, 10, 10], [20, 20, 40, 40]], float),
                "labels": np.array([1, 1, 2]), "scores": np.array([0.99, 0.9, 0.9])}
    r = C.evaluate_bbox(noisy, gts)
    assert 0.5 < r["AP"] < 1.0 and 0.5 < r["AP50"] < 1.0


@pytest.fixture(scope="module")
def coco_root(tmp_path_factory):
    spec = importlib.util.spec_from_file_location("mrcnn_train", os.path.join(HERE, "..", "examples", "ai",
                                                                              "maskrcnn_train.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    root = str(tmp_path_factory.mktemp("coco"))
    mod.main(["--coco-root", root, "--make-coco", "4"])
    return root, mod


def test_loader_geometry_and_flip(coco_root):
    root, _ = coco_root
    ds = C.CocoDetection(os.path.join(root, "train"), os.path.join(root, "annotations", "instances_train.json"))
    assert ds.num_classes == 3 and sorted(ds.cat_to_label) == [3, 7]
    plain = C.CocoLoader(ds, 2, min_size=160, max_size=256, workers=0, flip_prob=0.0)
    imgs, targets, sizes, ids, scales = next(iter(plain))
    assert imgs.shape[0] == 2 and imgs.shape[2] % 32 == 0 and imgs.shape[3] % 32 == 0
    for t, (h, w) in zip(targets, sizes):
        assert min(h, w) == 160 or max(h, w) == 256
        assert t["masks"].shape[1:] == imgs.shape[2:] and t["masks"].sum() > 0
        b = t["boxes"]
        assert (b[:, 2] <= w + 1e-3).all() and (b[:, 3] <= h + 1e-3).all()
        # each mask lies inside its box (polygon outlines of rectangles / triangles)
        for m, (x1, y1, x2, y2) in zip(t["masks"], b.tolist()):
            ys, xs = torch.nonzero(m, as_tuple=True)
            assert xs.min() >= x1 - 2 and xs.max() <= x2 + 2 and ys.min() >= y1 - 2 and ys.max() <= y2 + 2
    flipped = C.CocoLoader(ds, 2, min_size=160, max_size=256, workers=0, flip_prob=1.0)
    _, ft, fsizes, fids, _ = next(iter(flipped))
    assert fids == ids
    for t, f, (h, w) in zip(targets, ft, sizes):
        torch.testing.assert_close(f["boxes"][:, [0, 2]], w - t["boxes"][:, [2, 0]])
        torch.testing.assert_close(f["masks"][:, :h, :w], t["masks"][:, :h, :w].flip(-1))


def test_maskrcnn_entry_trains_and_evaluates_cpu(coco_root, monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    root, mod = coco_root
    r = mod.main(["--coco-root", root, "--batch", "2", "--min-size", "128", "--max-size", "192", "--max-iter", "2",
                  "--warmup-iters", "1", "--steps", "1", "--workers", "0", "--log-every", "1"])
    assert r["steps"] == 2 and all(math.isfinite(v) for v in r["losses"].values())
    assert set(r["bbox"]) == {"AP", "AP50", "AP75"} and 0.0 <= r["bbox"]["AP"] <= 1.0


def test_warmup_multistep_schedule():
    from cloudtik_amd.train.lr_scheduler import WarmupMultiStepScheduler

    class O:
        param_groups = [{"lr": 0.02}]
    s = WarmupMultiStepScheduler(O(), [4, 6], 0.1, 1 / 3, 2)
    lrs = [O.param_groups[0]["lr"]]
    for _ in range(7):
        s.step()
        lrs.append(O.param_groups[0]["lr"])
    assert lrs[0] == pytest.approx(0.02 / 3) and lrs[2] == pytest.approx(0.02)
    assert lrs[4] == pytest.approx(0.002) and lrs[6] == pytest.approx(0.0002)


def test_fixed_canvas_groups_by_orientation(tmp_path):
    """fixed_canvas: one padded canvas per orientation, batches never mix orientations, every
    eval image is still visited once, and train ranks yield equal batch counts."""
    import json
    from PIL import Image
    from cloudtik_amd.data.coco import CocoDetection, CocoLoader
    images, anns = [], []
    for i, (w, h) in enumerate([(200, 120), (120, 200), (210, 100), (100, 190), (220, 130), (180, 110), (90, 170)]):
        Image.new("RGB", (w, h), (i * 20, 40, 90)).save(tmp_path / f"{i}.jpg")
        images.append({"id": i + 1, "file_name": f"{i}.jpg", "width": w, "height": h})
        anns.append({"id": i + 1, "image_id": i + 1, "category_id": 1, "iscrowd": 0, "bbox": [5, 5, 40, 30],
                     "area": 1200.0, "segmentation": [[5, 5, 45, 5, 45, 35, 5, 35]]})
    ann = tmp_path / "ann.json"
    ann.write_text(json.dumps({"images": images, "annotations": anns, "categories": [{"id": 1, "name": "a"}]}))
    ds = CocoDetection(str(tmp_path), str(ann), train=False, with_masks=False)
    ld = CocoLoader(ds, 2, min_size=96, max_size=160, workers=0, fixed_canvas=True, drop_last=False)
    seen, shapes = [], set()
    for imgs, _, sizes, ids, _ in ld:
        shapes.add(tuple(imgs.shape[2:]))
        assert len({h >= w for h, w in sizes}) == 1 or len(sizes) == 1
        seen += list(ids)
    assert sorted(seen) == list(range(1, 8)) and shapes <= {(96, 160), (160, 96)}
    tr = CocoDetection(str(tmp_path), str(ann), train=True, with_masks=False)
    loaders = [CocoLoader(tr, 2, 96, 160, rank=r, world=2, workers=0, fixed_canvas=True) for r in range(2)]
    ids = [[i for _, _, _, b, _ in ld for i in b] for ld in loaders]
    assert len(ids[0]) // 2 == len(ids[1]) // 2 == len(loaders[0]) == len(loaders[1])
    assert all(len(x) == len(set(x)) for x in ids)            # no image twice within an epoch
    assert not set(ids[0]) & set(ids[1])                       # ranks see disjoint images
    assert len(ld) == sum(1 for _ in ld)                       # eval __len__ matches what it yields
