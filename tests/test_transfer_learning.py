"""Transfer learning (ai.modeling.transfer_learning) on CPU: image and text classifiers
fine-tune on learnable synthetic data, export / reload, pretrained-weight loading, and the
run.py workflow over an image folder.  Hub checkpoints cannot be fetched here, so accuracy
parity with the reference's pretrained models is unpinned."""
import os

import numpy as np
import pytest
import torch

from cloudtik_amd.modeling.transfer_learning import (HashTokenizer, ImageClassificationModel,
                                                     TextClassificationDataset, get_model, get_supported_models,
                                                     load_model, synthetic_image_dataset)


def test_factory_lists_models():
    s = get_supported_models()
    assert "resnet50" in s["image_classification"] and "bert-base-uncased" in s["text_classification"]
    with pytest.raises(ValueError):
        get_model("vgg16")


def test_image_classifier_finetune_export_reload(tmp_path):
    torch.manual_seed(0)
    full = synthetic_image_dataset(288, 3, image_size=32)
    ds, ev = torch.utils.data.random_split(full, [192, 96], generator=torch.Generator().manual_seed(0))
    m = get_model("resnet_tiny", use_case="image_classification", num_classes=3, freeze_backbone=False, device="cpu")
    hist = m.train(ds, epochs=3, batch_size=32, lr=3e-3, log_every=0)
    assert hist[-1]["loss"] < hist[0]["loss"]
    acc = m.evaluate(ev)["accuracy"]
    assert acc > 0.6, acc
    m.export(str(tmp_path / "img"))
    m2 = load_model(str(tmp_path / "img"), device="cpu")
    x = torch.stack([ev[i][0] for i in range(4)])
    torch.testing.assert_close(m.predict(x), m2.predict(x))


def test_frozen_backbone_only_trains_head(tmp_path):
    src = ImageClassificationModel("resnet_tiny", 5, freeze_backbone=False, device="cpu")
    torch.save(src.model.state_dict(), tmp_path / "pre.pt")
    m = ImageClassificationModel("resnet_tiny", 3, pretrained_path=str(tmp_path / "pre.pt"), device="cpu")
    torch.testing.assert_close(m.model.conv1.weight, src.model.conv1.weight)
    before = {n: p.detach().clone() for n, p in m.model.named_parameters()}
    m.train(synthetic_image_dataset(64, 3, image_size=32), epochs=1, batch_size=32, log_every=0)
    for n, p in m.model.named_parameters():
        changed = not torch.equal(p, before[n])
        assert changed == n.startswith("fc."), n


def test_text_classifier_learns_keywords(tmp_path):
    rng = np.random.default_rng(0)
    pos, neg = ["great", "good", "excellent", "love"], ["bad", "awful", "terrible", "hate"]
    filler = ["the", "movie", "was", "plot", "acting", "really", "quite"]
    texts, labels = [], []
    for _ in range(400):
        y = int(rng.integers(0, 2))
        words = list(rng.choice(filler, 6)) + [rng.choice(pos if y else neg)]
        rng.shuffle(words)
        texts.append(" ".join(words))
        labels.append(y)
    tok = HashTokenizer(vocab_size=512, max_length=16)
    ds = TextClassificationDataset(texts[:320], labels[:320], tok)
    ev = TextClassificationDataset(texts[320:], labels[320:], tok)
    m = get_model("bert-tiny", use_case="text_classification", num_classes=2, device="cpu")
    m.train(ds, epochs=4, batch_size=32, lr=1e-3, log_every=0)
    assert m.evaluate(ev)["accuracy"] > 0.85
    m.export(str(tmp_path / "txt"))
    m2 = load_model(str(tmp_path / "txt"), device="cpu")
    torch.testing.assert_close(m.predict(ev.ids[:4], ev.mask[:4]), m2.predict(ev.ids[:4], ev.mask[:4]))


def test_run_image_folder(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    for c, colour in (("cat", (200, 30, 30)), ("dog", (30, 30, 200))):
        os.makedirs(tmp_path / "data" / c)
        for i in range(12):
            a = np.clip(np.array(colour)[None, None] + rng.normal(0, 20, (40, 48, 3)), 0, 255).astype(np.uint8)
            Image.fromarray(a).save(tmp_path / "data" / c / f"{i}.png")
    from cloudtik_amd.modeling.transfer_learning import run as tl_run
    out = tl_run.main(["--model", "resnet_tiny", "--dataset-dir", str(tmp_path / "data"), "--image-size", "32",
                       "--epochs", "2", "--batch-size", "8", "--no-freeze", "--lr", "3e-3",
                       "--output-dir", str(tmp_path / "out"), "--device", "cpu", "--val-split", "0.25"])
    assert os.path.exists(out["export"]) and "eval_accuracy" in out["history"][-1]
