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


@pytest.mark.parametrize("flip", [False, True])
def test_image_ingest_kernel(cuda, flip):
    from cloudtik_amd import ops
    from cloudtik_amd.ops.vision import images_to_tensor_reference
    g = torch.Generator().manual_seed(1)
    imgs = torch.randint(0, 256, (5, 24, 36, 3), generator=g, dtype=torch.uint8)
    f = torch.tensor([1, 0, 1, 1, 0], dtype=torch.uint8) if flip else None
    got = ops.images_to_tensor(imgs.cuda(), None if f is None else f.cuda())
    assert got.dtype == torch.bfloat16 and got.shape == (5, 3, 24, 36)
    assert got.is_contiguous(memory_format=torch.channels_last)
    want = images_to_tensor_reference(imgs, f)
    torch.testing.assert_close(got.float().cpu(), want, rtol=1e-2, atol=2e-2)


def test_parquet_image_pipeline_gpu(cuda, tmp_path):
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, PYTHONPATH=os.getcwd())
    r = subprocess.run([sys.executable, "examples/ai/spark_parquet_resnet50.py", "--model", "small",
                        "--image-size", "64", "--batch-size", "64", "--data-path", str(tmp_path / "pq"),
                        "--epochs", "2", "--warmup", "2"], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["value"] > 0 and res["final_loss"] == res["final_loss"]
