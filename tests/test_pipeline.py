"""Spark -> Parquet -> loader pipeline on CPU (ETL writer, per-rank part assignment, image
ingest reference, ParquetImageLoader batches)."""
import numpy as np
import torch

from cloudtik_amd.data.pipeline import ParquetImageLoader, rank_parts, write_image_shards
from cloudtik_amd.ops.vision import images_to_tensor


def test_etl_and_loader(tmp_path):
    paths = write_image_shards(str(tmp_path), 100, 4, image_size=8, num_classes=5, engine="pyarrow", workers=2)
    assert len(paths) == 4
    assert rank_parts(str(tmp_path), 1, 2) == sorted(paths)[1::2]
    ld = ParquetImageLoader(rank_parts(str(tmp_path), 0, 2), 16, image_size=8, flip_prob=0.5, device="cpu")
    assert ld.num_rows == 50 and len(ld) == 3
    n = 0
    for x, y in ld:
        assert x.shape == (16, 3, 8, 8) and x.dtype == torch.float32 and y.dtype == torch.int64
        assert float(x.abs().max()) < 3.0
        n += 1
    assert n == 3
    ld.close()


def test_images_to_tensor_flip_reference():
    imgs = torch.arange(2 * 2 * 4 * 3, dtype=torch.uint8).reshape(2, 2, 4, 3)
    out = images_to_tensor(imgs, torch.tensor([1, 0]), mean=(0, 0, 0), std=(1, 1, 1))
    assert torch.allclose(out[0], (imgs[0].flip(1).float() / 255).permute(2, 0, 1))
    assert torch.allclose(out[1], (imgs[1].float() / 255).permute(2, 0, 1))
