"""ImageFolder JPEG pipeline (data/imagefolder.py): scan order, rank sharding, the
RandomResizedCrop / centre-crop geometry, pool == in-process decoding, normalised output."""
import numpy as np
import pytest
import torch


@pytest.fixture(scope="module")
def folder(tmp_path_factory):
    from PIL import Image
    root = tmp_path_factory.mktemp("imgs")
    rng = np.random.default_rng(0)
    for c in ("cat", "dog", "eel"):
        (root / c).mkdir()
        for i in range(6):
            w, h = int(rng.integers(40, 90)), int(rng.integers(40, 90))
            Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(root / c / f"{i}.jpg")
    (root / "dog" / "notes.txt").write_text("not an image")
    return str(root)


def test_scan_matches_imagefolder_order(folder):
    from cloudtik_amd.data.imagefolder import scan_image_folder
    samples, classes = scan_image_folder(folder)
    assert classes == ["cat", "dog", "eel"] and len(samples) == 18
    assert [c for _, c in samples] == [0] * 6 + [1] * 6 + [2] * 6


def test_train_batches_shapes_sharding_and_determinism(folder):
    from cloudtik_amd.data.imagefolder import ImageFolderLoader
    a = ImageFolderLoader(folder, 4, train=True, image_size=32, rank=0, world=2, workers=0, seed=3)
    b = ImageFolderLoader(folder, 4, train=True, image_size=32, rank=1, world=2, workers=0, seed=3)
    assert len(a) == len(b) == 2
    assert not set(a._indices()) & set(b._indices())
    xs = [(x, y) for x, y in a]
    assert xs[0][0].shape == (4, 3, 32, 32) and xs[0][1].dtype == torch.int64
    again = [(x, y) for x, y in a]
    torch.testing.assert_close(xs[0][0], again[0][0])          # same epoch -> same crops
    a.set_epoch(1)
    other = [(x, y) for x, y in a]
    assert not torch.equal(xs[0][0], other[0][0])               # new epoch -> new permutation / crops
    # normalised range (ImageNet mean/std)
    assert xs[0][0].min() > -2.2 and xs[0][0].max() < 2.7


def test_pool_matches_in_process(folder):
    from cloudtik_amd.data.imagefolder import ImageFolderLoader
    kw = dict(train=True, image_size=24, seed=5, flip_prob=0.0)
    serial = [x for x, _ in ImageFolderLoader(folder, 3, workers=0, **kw)]
    ld = ImageFolderLoader(folder, 3, workers=2, prefetch=2, **kw)
    pooled = [x for x, _ in ld]
    ld.close()
    assert len(serial) == len(pooled) == 6
    for s, p in zip(serial, pooled):
        torch.testing.assert_close(s, p)


def test_eval_center_crop_geometry(folder):
    from PIL import Image
    from cloudtik_amd.data.imagefolder import ImageFolderLoader, scan_image_folder, _decode_batch
    samples, _ = scan_image_folder(folder)
    p = samples[0][0]
    out = _decode_batch(([p], [0], 16, False, 20))[0]
    with Image.open(p) as im:
        im = im.convert("RGB")
        w, h = im.size
        sc = 20 / min(w, h)
        nw, nh = max(16, round(w * sc)), max(16, round(h * sc))
        im = im.resize((nw, nh), Image.BILINEAR)
        l, t = (nw - 16) // 2, (nh - 16) // 2
        ref = np.asarray(im.crop((l, t, l + 16, t + 16)))
    assert np.array_equal(out, ref)
    ev = ImageFolderLoader(folder, 5, train=False, image_size=16, workers=0)
    labels = torch.cat([y for _, y in ev])
    assert labels.tolist() == [c for _, c in samples][:15]      # eval keeps file order


def test_random_resized_crop_box_bounds():
    import random
    from cloudtik_amd.data.imagefolder import random_resized_crop_box
    rng = random.Random(0)
    for _ in range(200):
        w, h = rng.randint(10, 500), rng.randint(10, 500)
        l, t, cw, ch = random_resized_crop_box(w, h, rng)
        assert 0 <= l and 0 <= t and cw > 0 and ch > 0 and l + cw <= w and t + ch <= h
