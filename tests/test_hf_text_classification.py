"""Hugging Face text classification on the native BERT (modeling/transfer_learning/hugging_face.py)
and the dataset factory (dataset_factory.py); reference text_classification/pytorch/hugging_face/
text_classification_model.py and dataset_factory.py:100.

* weight-mapped parity: a random ``transformers.BertForSequenceClassification`` (fp32, dropout 0,
  padded attention mask) saved with ``save_pretrained`` and loaded by the native model gives the
  same logits, loss and (mapped) parameter gradients;
* ``export`` writes an HF checkpoint that ``transformers`` reloads with identical logits;
* fine-tuning through the framework Trainer learns a separable toy task;
* datasets: local csv files via ``datasets`` with an HF WordPiece tokenizer built from a local
  vocab, ``save_to_disk`` directories, and the factory's folder / csv layouts."""
import os

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
pytest.importorskip("datasets")

from cloudtik_amd.modeling.transfer_learning import hugging_face as HF  # noqa: E402
from cloudtik_amd.modeling.transfer_learning.dataset_factory import get_dataset, load_dataset  # noqa: E402

WORDS = ["good", "great", "fine", "love", "bad", "awful", "poor", "hate", "the", "movie", "was", "a", "plot"]


def _hf_checkpoint(tmp_path, num_labels=3, L=2):
    cfg = transformers.BertConfig(vocab_size=120, hidden_size=64, num_hidden_layers=L, num_attention_heads=4,
                                  intermediate_size=128, max_position_embeddings=64, hidden_dropout_prob=0.0,
                                  attention_probs_dropout_prob=0.0, num_labels=num_labels)
    torch.manual_seed(0)
    hf = transformers.BertForSequenceClassification(cfg).float().eval()
    d = str(tmp_path / "ckpt")
    hf.save_pretrained(d, safe_serialization=True)
    return hf, d


def _batch(B=4, S=16, V=120):
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1, V, (B, S), generator=g)
    mask = torch.ones(B, S, dtype=torch.long)
    mask[1, 10:] = 0
    mask[3, 5:] = 0
    tt = torch.zeros(B, S, dtype=torch.long)
    tt[:, S // 2:] = 1
    y = torch.tensor([0, 2, 1, 2])
    return ids, mask, tt, y


def test_weight_mapped_parity_with_transformers(tmp_path):
    hf, d = _hf_checkpoint(tmp_path)
    m = HF.HuggingFaceTextClassificationModel(d, num_classes=3, device="cpu", dtype=torch.float32)
    ours = m.model.eval()
    ids, mask, tt, y = _batch()
    ref = hf(input_ids=ids, attention_mask=mask, token_type_ids=tt, labels=y)
    out = ours(ids, mask, tt)
    torch.testing.assert_close(out, ref.logits, rtol=1e-4, atol=1e-4)
    loss = torch.nn.functional.cross_entropy(out, y)
    torch.testing.assert_close(loss, ref.loss, rtol=1e-5, atol=1e-5)
    ref.loss.backward()
    loss.backward()
    hf_grads = {n: p.grad for n, p in hf.named_parameters()}
    mine = dict(ours.named_parameters())
    for name, theirs in HF.weight_map(2):
        g_ref = torch.cat([hf_grads[t] for t in theirs]) if len(theirs) > 1 else hf_grads[theirs[0]]
        g = mine[name].grad
        if name == "bert.word_embeddings":
            g = g[: g_ref.shape[0]]
        torch.testing.assert_close(g, g_ref.view_as(g), rtol=1e-3, atol=1e-5, msg=name)


def test_export_roundtrip_opens_in_transformers(tmp_path):
    hf, d = _hf_checkpoint(tmp_path)
    m = HF.HuggingFaceTextClassificationModel(d, num_classes=3, device="cpu", dtype=torch.float32,
                                              classes=["neg", "neu", "pos"])
    with torch.no_grad():
        m.model.classifier.weight.mul_(1.5)            # a "fine-tuned" change that must round-trip
    out_dir = m.export(str(tmp_path / "export"))
    back = transformers.BertForSequenceClassification.from_pretrained(out_dir).float().eval()
    assert back.config.id2label[2] == "pos"
    ids, mask, tt, _ = _batch()
    torch.testing.assert_close(back(input_ids=ids, attention_mask=mask, token_type_ids=tt).logits,
                               m.model.eval()(ids, mask, tt), rtol=1e-4, atol=1e-4)
    again = HF.HuggingFaceTextClassificationModel.load(out_dir, device="cpu")
    assert again.classes == ["neg", "neu", "pos"]
    torch.testing.assert_close(again.model.eval()(ids, mask, tt), m.model(ids, mask, tt), rtol=1e-5, atol=1e-5)


def _vocab_tokenizer(tmp_path):
    vocab = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"] + WORDS
    vf = tmp_path / "vocab.txt"
    vf.write_text("\n".join(vocab) + "\n")
    return transformers.BertTokenizerFast(vocab=str(vf), do_lower_case=True), len(vocab)


def _csv_dataset(tmp_path, n=96):
    rng = np.random.default_rng(0)
    d = tmp_path / "reviews"
    d.mkdir()
    rows = ["text,label"]
    for i in range(n):
        pos = i % 2 == 0
        pool = WORDS[:4] if pos else WORDS[4:8]
        words = list(rng.choice(pool, 3)) + list(rng.choice(WORDS[8:], 3))
        rng.shuffle(words)
        rows.append(f"{' '.join(words)},{'positive' if pos else 'negative'}")
    (d / "train.csv").write_text("\n".join(rows) + "\n")
    return str(d)


def test_hf_dataset_from_local_csv_and_finetune(tmp_path):
    tok, V = _vocab_tokenizer(tmp_path)
    ds = get_dataset(_csv_dataset(tmp_path), "text_classification", "pytorch", "reviews")
    assert isinstance(ds, HF.HuggingFaceTextClassificationDataset)
    assert ds.class_names == ["negative", "positive"] and len(ds) == 96
    ds.preprocess(tok, batch_size=16, max_length=16)
    ds.shuffle_split(train_pct=0.75, val_pct=0.25, seed=0)
    first = ds.train_subset[0]
    assert first["input_ids"].shape == (16,) and int(first["input_ids"][0]) == tok.cls_token_id
    assert len(ds.train_subset) == 72 and len(ds.validation_subset) == 24
    b = next(iter(ds.train_loader))
    assert b["input_ids"].shape == (16, 16) and b["label"].shape == (16,)
    # a small random-init BERT of the catalogue's family learns the separable task
    hf_cfg = transformers.BertConfig(vocab_size=V, hidden_size=32, num_hidden_layers=1, num_attention_heads=2,
                                     intermediate_size=64, max_position_embeddings=32, num_labels=2)
    ck = str(tmp_path / "tiny")
    torch.manual_seed(0)
    transformers.BertForSequenceClassification(hf_cfg).save_pretrained(ck)
    tok.save_pretrained(ck)
    m = HF.HuggingFaceTextClassificationModel(ck, num_classes=2, device="cpu", dtype=torch.float32,
                                              hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    assert m.tokenizer is not None
    hist = m.train(ds, epochs=12, batch_size=16, lr=3e-3, log_every=0)
    assert hist[-1]["loss"] < hist[0]["loss"]
    assert m.evaluate(ds)["accuracy"] >= 0.9
    pred = m.predict(["good great love the movie", "awful bad hate the plot"])
    assert pred.tolist() == [1, 0]


def test_hf_dataset_from_save_to_disk(tmp_path):
    import datasets
    d = datasets.DatasetDict({"train": datasets.Dataset.from_dict({"sentence": ["a b", "c d", "e f", "g h"],
                                                                   "label": [0, 1, 0, 1]}),
                              "validation": datasets.Dataset.from_dict({"sentence": ["x"], "label": [1]})})
    path = str(tmp_path / "saved")
    d.save_to_disk(path)
    ds = load_dataset(path, "text_classification", "pytorch", source="hugging_face", split=["train", "validation"])
    assert len(ds) == 5 and ds.text_column == "sentence" and ds.class_names == ["0", "1"]
    ds.preprocess(None, batch_size=2, max_length=8)            # hash tokenizer fallback
    ds.shuffle_split(0.6, 0.4, seed=1)
    assert len(ds.train_subset) == 3


def test_dataset_factory_user_layouts(tmp_path):
    from PIL import Image
    for split in ("train", "validation"):
        for c in ("cat", "dog"):
            p = tmp_path / "pets" / split / c
            p.mkdir(parents=True)
            for i in range(2):
                Image.fromarray(np.full((8, 8, 3), 40 * i, dtype=np.uint8)).save(p / f"{i}.jpg")
    img = load_dataset(str(tmp_path / "pets"), "image_classification", "pytorch", image_size=8)
    assert img.class_names == ["cat", "dog"] and len(img.train_subset) == 4 and len(img.validation_subset) == 4
    txt_dir = tmp_path / "txt"
    txt_dir.mkdir()
    (txt_dir / "data.csv").write_text("spam,buy now\nham,see you\nspam,win cash\n")
    txt = load_dataset(str(txt_dir), "text_classification", "pytorch")
    assert txt.class_names == ["ham", "spam"] and len(txt) == 3
    assert int(txt.dataset[0]["label"]) == 1
    with pytest.raises(NotImplementedError):
        load_dataset(str(txt_dir), "text_classification", "tensorflow")
    with pytest.raises(ValueError):
        load_dataset(str(txt_dir), "", "pytorch")
