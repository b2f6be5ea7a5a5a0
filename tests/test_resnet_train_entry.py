"""ResNet-50 training entry (examples/ai/resnet50_train.py) on a synthetic JPEG folder, CPU."""
import importlib.util
import math
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def test_resnet50_train_entry_runs_and_evaluates(tmp_path, monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    spec = importlib.util.spec_from_file_location("rn50_train", os.path.join(HERE, "..", "examples", "ai",
                                                                             "resnet50_train.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    root = str(tmp_path / "imgs")
    mod.main(["--data", root, "--make-folder", "2x4"])
    assert sorted(os.listdir(os.path.join(root, "train"))) == ["n00000000", "n00000001"]
    r = mod.main(["--data", root, "--epochs", "1", "--batch", "4", "--image-size", "32", "--workers", "0",
                  "--log-every", "1", "--ckpt-dir", str(tmp_path / "ck")])
    assert r["steps"] == 2 and math.isfinite(r["loss"])
    assert 0.0 <= r["val_top1"] <= 1.0 and r["val_top5"] == 1.0          # 2 classes: top-5 always hits
    assert os.listdir(tmp_path / "ck")
