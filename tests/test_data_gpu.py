"""Native loader in device mode: pinned slots -> hipMemcpyAsync on a side stream."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_native_loader_device(cuda, tmp_path):
    from cloudtik_amd.data import NativeLoader
    n = 10000
    x = np.random.rand(n, 3, 32, 32).astype(np.float32)
    y = np.arange(n, dtype=np.int64)
    L = NativeLoader({"x": x, "y": y}, 256, shuffle=True, seed=1, device=cuda, num_workers=4, prefetch=4)
    seen = []
    xt = torch.from_numpy(x).to(cuda)
    for b in L:
        assert b["x"].is_cuda and b["x"].shape[1:] == (3, 32, 32)
        # consumer-stream work right after next(): must observe the copied data
        assert torch.equal(b["x"], xt[b["y"]])
        seen.append(b["y"].cpu())
    allidx = torch.cat(seen)
    assert allidx.numel() == n and torch.unique(allidx).numel() == n
    L.set_epoch(1)
    first = next(iter(L))["y"].cpu()
    assert not torch.equal(first, seen[0])
    L.close()


def test_parquet_to_gpu(cuda, tmp_path):
    from cloudtik_amd.data import ParquetDataLoader, write_parquet
    imgs = np.random.randint(0, 255, (777, 3, 8, 8), dtype=np.uint8)
    write_parquet(str(tmp_path / "part-0.parquet"), {"image": imgs[:400], "label": np.arange(400)})
    write_parquet(str(tmp_path / "part-1.parquet"), {"image": imgs[400:], "label": np.arange(400, 777)})
    P = ParquetDataLoader(str(tmp_path), 128, shapes={"image": (3, 8, 8)}, device=cuda, shuffle=False)
    got = torch.cat([b["image"].cpu() for b in P])
    assert torch.equal(got, torch.from_numpy(imgs))
