"""Image anomaly detection (reference transfer_learning/image_anomaly_detection): PCA on
backbone features of good images scores synthetic defects above good images; the CutPaste
and SimSiam self-supervised adaptations train with finite losses (CPU, tiny backbone)."""
import numpy as np
import pytest
import torch


def _make(root, n_good=24, n_test_good=8, n_bad=8, size=32, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:size, 0:size]

    def good_img():
        ph = rng.uniform(0, 6.28)
        base = 120 + 40 * np.sin(xx / 3.0 + ph) + 20 * np.cos(yy / 4.0)
        return np.stack([base, base * 0.9, base * 0.8], -1) + rng.normal(0, 3, (size, size, 3))

    def save(arr, path):
        path.parent.mkdir(parents=True, exist_ok=True)
        Image.fromarray(np.clip(arr, 0, 255).astype(np.uint8)).save(path)
    for i in range(n_good):
        save(good_img(), root / "train" / "good" / f"{i}.png")
    for i in range(n_test_good):
        save(good_img(), root / "test" / "good" / f"{i}.png")
    for i in range(n_bad):
        a = good_img()
        y0, x0 = rng.integers(2, size - 12, 2)
        a[y0:y0 + 10, x0:x0 + 10] = rng.uniform(0, 255, 3)       # a solid-colour defect
        save(a, root / "test" / "scratch" / f"{i}.png")


def test_pca_scores_defects_higher(tmp_path):
    from cloudtik_amd.modeling.transfer_learning.anomaly_detection import AnomalyImageFolder, ImageAnomalyDetectionModel
    _make(tmp_path)
    torch.manual_seed(0)
    m = ImageAnomalyDetectionModel("resnet_tiny", layer_name="layer2", device="cpu")
    info = m.train(AnomalyImageFolder(str(tmp_path), "train", 32), batch_size=8)
    assert info["train_images"] == 24 and info["pca_components"] >= 1
    res = m.evaluate(AnomalyImageFolder(str(tmp_path), "test", 32))
    assert res["images"] == 16 and res["defective"] == 8
    assert res["auroc"] > 0.8, res
    x = torch.stack([AnomalyImageFolder(str(tmp_path), "test", 32)[i][0] for i in range(2)])
    assert m.predict(x).shape == (2,)
    assert set(m.predict(x, threshold=0.0, return_type="class").tolist()) <= {0, 1}
    from cloudtik_amd.modeling.transfer_learning.model_factory import get_model, load_model
    m.save(str(tmp_path / "out"))
    m2 = load_model(str(tmp_path / "out"), device="cpu")
    assert torch.allclose(m2.predict(x), m.predict(x))
    assert type(get_model("resnet_tiny", use_case="image_anomaly_detection", device="cpu")).__name__ == \
        "ImageAnomalyDetectionModel"


@pytest.mark.parametrize("method", ["cutpaste", "simsiam"])
def test_self_supervised_adaptation_runs(tmp_path, method):
    from cloudtik_amd.modeling.transfer_learning.anomaly_detection import AnomalyImageFolder, ImageAnomalyDetectionModel
    _make(tmp_path, n_good=8, n_test_good=2, n_bad=2)
    m = ImageAnomalyDetectionModel("resnet_tiny", layer_name="layer2", device="cpu")
    info = m.train(AnomalyImageFolder(str(tmp_path), "train", 32), batch_size=4, method=method, epochs=2)
    assert len(info["ssl_losses"]) == 2 and all(np.isfinite(info["ssl_losses"]))
    assert "auroc" in m.evaluate(AnomalyImageFolder(str(tmp_path), "test", 32))


def test_cutpaste_changes_a_patch_only():
    from cloudtik_amd.modeling.transfer_learning.anomaly_detection import cutpaste
    x = torch.zeros(3, 64, 64)
    x[:, :, :32] = 1.0
    y = cutpaste(x, torch.Generator().manual_seed(1))
    changed = (y != x).any(0).float().mean().item()
    assert 0 < changed < 0.2
