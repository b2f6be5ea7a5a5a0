"""Native loader (host mode) and the Parquet path on CPU."""
import numpy as np
import pytest
import torch


@pytest.mark.parametrize("world", [1, 3])
@pytest.mark.parametrize("drop_last", [False, True])
def test_loader_shards_cover_dataset(world, drop_last):
    from cloudtik_amd.data import NativeLoader
    n, B = 1000, 64
    x = np.arange(n * 3, dtype=np.float32).reshape(n, 3)
    y = np.arange(n)
    seen = []
    for r in range(world):
        L = NativeLoader({"x": x, "y": y}, B, shuffle=True, seed=5, rank=r, world=world, device="cpu",
                         num_workers=3, drop_last=drop_last)
        for b in L:
            assert (b["x"][:, 0].numpy() == b["y"].numpy() * 3).all()
            seen += b["y"].tolist()
        L.close()
    expect = (n // B // world) * world * B if drop_last else n
    assert len(seen) == expect and len(set(seen)) == expect


def test_loader_epochs_reshuffle_and_repeat():
    from cloudtik_amd.data import NativeLoader
    L = NativeLoader({"y": np.arange(256)}, 32, shuffle=True, seed=1, device="cpu")
    e0 = torch.cat([b["y"] for b in L])
    e0b = torch.cat([b["y"] for b in L])       # same epoch again
    L.set_epoch(1)
    e1 = torch.cat([b["y"] for b in L])
    assert torch.equal(e0, e0b) and not torch.equal(e0, e1)
    assert sorted(e1.tolist()) == list(range(256))


def test_parquet_roundtrip(tmp_path):
    from cloudtik_amd.data import ParquetDataLoader, read_parquet_columns, write_parquet
    imgs = np.random.randint(0, 255, (300, 2, 4, 4), dtype=np.uint8)
    write_parquet(str(tmp_path / "d" / "p0.parquet"), {"img": imgs[:100], "label": np.arange(100)})
    write_parquet(str(tmp_path / "d" / "p1.parquet"), {"img": imgs[100:], "label": np.arange(100, 300)})
    cols = read_parquet_columns(str(tmp_path / "d"), shapes={"img": (2, 4, 4)})
    assert cols["img"].shape == (300, 2, 4, 4) and (cols["img"] == imgs).all()
    P = ParquetDataLoader(str(tmp_path / "d"), 64, shapes={"img": (2, 4, 4)}, device="cpu", shuffle=False)
    got = torch.cat([b["img"] for b in P])
    assert torch.equal(got, torch.from_numpy(imgs))
