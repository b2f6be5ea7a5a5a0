"""BERT pretraining entry (examples/ai/bert_pretrain.py): synthetic MLPerf-layout shards ->
native loader -> LAMB + warmup/poly-decay -> checkpoint -> resume, on CPU."""
import importlib.util
import math
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _load():
    spec = importlib.util.spec_from_file_location("bert_pretrain", os.path.join(HERE, "..", "examples", "ai",
                                                                               "bert_pretrain.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_bert_pretrain_shards_train_and_resume(tmp_path, monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    bp = _load()
    data = str(tmp_path / "shards")
    common = ["--data-dir", data, "--config", "tiny", "--seq", "32", "--max-pred", "5"]
    bp.main(common + ["--make-shards", "2", "--shard-rows", "48"])
    assert len(os.listdir(data)) == 2
    ck = str(tmp_path / "ckpt")
    r1 = bp.main(common + ["--batch", "8", "--max-steps", "3", "--total-steps", "10", "--warmup-proportion", "0.2",
                           "--ckpt-dir", ck, "--ckpt-every", "1", "--log-every", "1", "--eval-dir", data])
    assert r1["steps"] == 3 and math.isfinite(r1["final_loss"]) and r1["eval"]["loss"] > 0
    r2 = bp.main(common + ["--batch", "8", "--max-steps", "5", "--total-steps", "10", "--ckpt-dir", ck,
                           "--ckpt-every", "1", "--log-every", "1"])
    assert r2["steps"] == 5                                # resumed at step 3, ran 2 more


def test_padding_mask_slots_are_ignored():
    import torch
    bp = _load()
    b = {"input_ids": torch.ones(2, 8, dtype=torch.int32), "segment_ids": torch.zeros(2, 8, dtype=torch.int8),
         "input_mask": torch.ones(2, 8, dtype=torch.int8),
         "masked_lm_positions": torch.tensor([[1, 3, 0], [2, 0, 0]], dtype=torch.int32),
         "masked_lm_ids": torch.tensor([[7, 9, 0], [4, 0, 0]], dtype=torch.int32),
         "next_sentence_labels": torch.tensor([0, 1], dtype=torch.int8)}
    m = bp.to_model_batch(b)
    assert m["masked_lm_ids"].tolist() == [[7, 9, -100], [4, -100, -100]]
    assert all(v.dtype == torch.long for v in m.values())
