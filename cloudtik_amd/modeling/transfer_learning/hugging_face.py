"""Hugging Face text classification on the framework's BERT kernels (reference
modeling/transfer_learning/text_classification/pytorch/hugging_face/text_classification_model.py
and text_classification_dataset.py, common/pytorch/hugging_face/{model,dataset}.py).

The reference fine-tunes ``transformers.AutoModelForSequenceClassification`` as is (eager
PyTorch, or the HF Trainer).  Here the HF checkpoint is the interchange format, not the compute
path:

* ``HuggingFaceTextClassificationModel`` reads a local HF checkpoint directory (or, with no
  network to reach the hub, builds the named architecture -- ``HF_MODELS`` -- from its config
  with random weights), maps the weights one to one onto ``models.bert.BertModel`` + a linear
  classifier (fused HIP attention / LayerNorm / bias-GELU kernels, flat-buffer fused AdamW,
  bucketed data parallelism through ``train.trainer.Trainer``) and ``export`` writes a
  standard HF checkpoint back (``save_pretrained``: config + safetensors, tokenizer files if one
  was loaded), so the fine-tuned model opens in ``transformers`` unchanged;
* ``HuggingFaceTextClassificationDataset`` wraps ``datasets``: a local dataset directory
  saved by ``save_to_disk``, local csv / json / parquet files, or a named dataset already in
  the local HF cache; ``preprocess`` tokenizes with an HF tokenizer (a local tokenizer
  directory or vocab file; the hash tokenizer otherwise) and ``shuffle_split`` /
  ``train_subset`` / ``validation_subset`` / loaders follow the reference dataset API.

Weight mapping (HF name -> ours): ``bert.embeddings.*`` -> word/position/token-type tables and
``emb_ln_*`` (vocab rows padded to a multiple of 64); per layer the query/key/value projections
are concatenated into ``qkv_*``; ``attention.output.dense`` -> ``out_*``;
``attention.output.LayerNorm`` -> ``ln1_*``; ``intermediate.dense`` -> ``ffn1_*``;
``output.dense`` -> ``ffn2_*``; ``output.LayerNorm`` -> ``ln2_*``; ``bert.pooler.dense`` ->
``pooler_*``; ``classifier`` -> ``classifier``.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset

from cloudtik_amd.models.bert import BertConfig

from .image_classification import _default_device
from .text_classification import BertClassifier

# the reference's text_classification_models.json catalogue (architecture dims; no hub access)
HF_MODELS: Dict[str, Dict[str, Any]] = {
    "bert-base-uncased": dict(vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                              intermediate_size=3072),
    "bert-base-cased": dict(vocab_size=28996, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                            intermediate_size=3072),
    "bert-large-uncased": dict(vocab_size=30522, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                               intermediate_size=4096),
    "clinical-bert": dict(vocab_size=28996, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                          intermediate_size=3072),       # emilyalsentzer/Bio_ClinicalBERT
}


def _transformers():
    try:
        import transformers
    except ImportError as e:  # pragma: no cover - depends on the image
        raise RuntimeError("the Hugging Face path needs the `transformers` package") from e
    return transformers


# ------------------------------------------------------------------ configs and weights
def bert_config_from_hf(hf_cfg, **overrides) -> BertConfig:
    if getattr(hf_cfg, "model_type", "bert") != "bert":
        raise ValueError(f"only BERT-architecture checkpoints map onto the native encoder, got {hf_cfg.model_type!r}")
    if getattr(hf_cfg, "hidden_act", "gelu") not in ("gelu", "gelu_python"):
        raise ValueError(f"activation {hf_cfg.hidden_act!r} is not the erf GELU of the native kernels")
    d = dict(vocab_size=hf_cfg.vocab_size, hidden_size=hf_cfg.hidden_size, num_hidden_layers=hf_cfg.num_hidden_layers,
             num_attention_heads=hf_cfg.num_attention_heads, intermediate_size=hf_cfg.intermediate_size,
             hidden_dropout_prob=hf_cfg.hidden_dropout_prob,
             attention_probs_dropout_prob=hf_cfg.attention_probs_dropout_prob,
             max_position_embeddings=hf_cfg.max_position_embeddings, type_vocab_size=hf_cfg.type_vocab_size,
             layer_norm_eps=hf_cfg.layer_norm_eps, initializer_range=hf_cfg.initializer_range)
    d.update(overrides)
    return BertConfig(**d)


def hf_config_from_bert(cfg: BertConfig, num_labels: int, id2label: Optional[Dict[int, str]] = None):
    t = _transformers()
    kw = dict(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, num_hidden_layers=cfg.num_hidden_layers,
              num_attention_heads=cfg.num_attention_heads, intermediate_size=cfg.intermediate_size,
              hidden_dropout_prob=cfg.hidden_dropout_prob,
              attention_probs_dropout_prob=cfg.attention_probs_dropout_prob,
              max_position_embeddings=cfg.max_position_embeddings, type_vocab_size=cfg.type_vocab_size,
              layer_norm_eps=cfg.layer_norm_eps, initializer_range=cfg.initializer_range, hidden_act="gelu",
              num_labels=num_labels)
    if id2label:
        kw.update(id2label={int(k): v for k, v in id2label.items()}, label2id={v: int(k) for k, v in id2label.items()})
    return t.BertConfig(**kw)


def _layer_map(i: int):
    p, q = f"bert.encoder.layer.{i}.", f"bert.layers.{i}."
    out = []
    for kind in ("weight", "bias"):
        out += [(q + f"out_{kind}", [p + f"attention.output.dense.{kind}"]),
                (q + f"ln1_{kind}", [p + f"attention.output.LayerNorm.{kind}"]),
                (q + f"ffn1_{kind}", [p + f"intermediate.dense.{kind}"]),
                (q + f"ffn2_{kind}", [p + f"output.dense.{kind}"]),
                (q + f"ln2_{kind}", [p + f"output.LayerNorm.{kind}"]),
                (q + f"qkv_{kind}", [p + f"attention.self.{n}.{kind}" for n in ("query", "key", "value")])]
    return out


def weight_map(num_layers: int, with_classifier: bool = True):
    """[(our parameter name, [HF tensor names concatenated along dim 0])]."""
    m = [("bert.word_embeddings", ["bert.embeddings.word_embeddings.weight"]),
         ("bert.position_embeddings", ["bert.embeddings.position_embeddings.weight"]),
         ("bert.token_type_embeddings", ["bert.embeddings.token_type_embeddings.weight"]),
         ("bert.emb_ln_weight", ["bert.embeddings.LayerNorm.weight"]),
         ("bert.emb_ln_bias", ["bert.embeddings.LayerNorm.bias"]),
         ("bert.pooler_weight", ["bert.pooler.dense.weight"]),
         ("bert.pooler_bias", ["bert.pooler.dense.bias"])]
    for i in range(num_layers):
        m += _layer_map(i)
    if with_classifier:
        m += [("classifier.weight", ["classifier.weight"]), ("classifier.bias", ["classifier.bias"])]
    return m


@torch.no_grad()
def load_hf_state(model: BertClassifier, hf_state: Dict[str, torch.Tensor], strict: bool = True):
    """Copy an HF BertForSequenceClassification state dict into ``model`` (padding vocab rows
    stay zero).  ``strict=False`` skips a missing / differently shaped classifier head (new
    label set)."""
    mine = dict(model.named_parameters())
    for ours, theirs in weight_map(model.bert.cfg.num_hidden_layers):
        if not all(t in hf_state for t in theirs):
            if strict or not ours.startswith("classifier"):
                raise KeyError(f"checkpoint lacks {theirs}")
            continue
        src = torch.cat([hf_state[t] for t in theirs]) if len(theirs) > 1 else hf_state[theirs[0]]
        dst = mine[ours]
        if ours.startswith("classifier") and src.shape != dst.shape and not strict:
            continue
        if ours == "bert.word_embeddings":
            dst.zero_()
            dst[: src.shape[0]].copy_(src)
        else:
            dst.copy_(src.to(dst.dtype).view_as(dst))


@torch.no_grad()
def to_hf_state(model: BertClassifier) -> Dict[str, torch.Tensor]:
    """The inverse of ``load_hf_state`` (fp32, contiguous, vocab padding dropped)."""
    cfg = model.bert.cfg
    mine = dict(model.named_parameters())
    out: Dict[str, torch.Tensor] = {}
    for ours, theirs in weight_map(cfg.num_hidden_layers):
        t = mine[ours].detach().float().cpu()
        if ours == "bert.word_embeddings":
            t = t[: cfg.vocab_size]
        if len(theirs) == 1:
            out[theirs[0]] = t.contiguous()
        else:
            for name, part in zip(theirs, t.chunk(len(theirs))):
                out[name] = part.contiguous()
    return out


# ------------------------------------------------------------------ model
class HuggingFaceTextClassificationModel:
    """Fine-tune / evaluate / predict / export an HF BERT sequence classifier on the native
    kernels (API of the reference's PyTorch HF ``TextClassificationModel``)."""

    use_case = "text_classification"

    def __init__(self, model_name_or_path: str = "bert-base-uncased", num_classes: int = 2, device=None,
                 dtype: Optional[torch.dtype] = None, classes: Optional[List[str]] = None,
                 freeze_encoder: bool = False, **config_overrides):
        t = _transformers()
        self.model_name = model_name_or_path
        self.device = torch.device(device) if device else _default_device()
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.tokenizer = None
        hf_state = None
        if os.path.isdir(model_name_or_path):
            hf_cfg = t.AutoConfig.from_pretrained(model_name_or_path, local_files_only=True)
            hf_state = self._read_checkpoint(model_name_or_path)
            try:
                self.tokenizer = t.AutoTokenizer.from_pretrained(model_name_or_path, local_files_only=True)
            except Exception:  # noqa: BLE001 - a checkpoint without tokenizer files
                self.tokenizer = None
            if classes is None and getattr(hf_cfg, "id2label", None) and len(hf_cfg.id2label) == num_classes:
                classes = [hf_cfg.id2label[i] for i in range(num_classes)]
        elif model_name_or_path in HF_MODELS:
            hf_cfg = t.BertConfig(**HF_MODELS[model_name_or_path])     # no hub: architecture only
        else:
            raise ValueError(f"{model_name_or_path!r} is neither a local HF checkpoint directory nor one of "
                             f"{sorted(HF_MODELS)}")
        self.cfg = bert_config_from_hf(hf_cfg, **config_overrides)
        self.num_classes, self.classes = num_classes, classes
        self.model = BertClassifier(self.cfg, num_classes, device=self.device, dtype=self.dtype)
        if hf_state is not None:
            load_hf_state(self.model, {k: v.to(self.device) for k, v in hf_state.items()}, strict=False)
        if freeze_encoder:
            for p in self.model.bert.parameters():
                p.requires_grad_(False)
        self.history: List[Dict[str, float]] = []

    @staticmethod
    def _read_checkpoint(path: str) -> Dict[str, torch.Tensor]:
        st = os.path.join(path, "model.safetensors")
        if os.path.exists(st):
            from safetensors.torch import load_file
            sd = load_file(st)
        else:
            sd = torch.load(os.path.join(path, "pytorch_model.bin"), map_location="cpu", weights_only=True)
        # BertModel / BertForPreTraining checkpoints name the encoder without the "bert." prefix
        if not any(k.startswith("bert.") for k in sd):
            sd = {("bert." + k if not k.startswith("classifier") else k): v for k, v in sd.items()}
        return sd

    @staticmethod
    def _step(model, batch):
        out = model(batch["input_ids"], batch.get("attention_mask"), batch.get("token_type_ids"))
        y = batch["label"]
        loss = F.cross_entropy(out.float(), y)
        return loss, {"loss": loss.detach(), "accuracy": (out.argmax(-1) == y).float().mean()}

    def train(self, dataset, epochs: int = 1, batch_size: int = 32, lr: float = 2e-5, eval_dataset=None,
              weight_decay: float = 0.01, checkpoint_dir: Optional[str] = None, seed: int = 0,
              max_steps: Optional[int] = None, log_every: int = 50, warmup_steps: int = 0,
              distributed: bool = False, nnodes: int = 1, nproc_per_node: int = 1, hosts: Optional[str] = None,
              hostfile: Optional[str] = None, shared_dir: Optional[str] = None, launcher: Optional[str] = None):
        """Fine-tune with the framework Trainer (data parallel when launched with several
        ranks).  ``dataset`` is a torch Dataset of dicts or a HuggingFaceTextClassificationDataset.
        ``distributed=True`` launches the ranks itself (modeling/transfer_learning/distributed.py)."""
        if distributed:
            from cloudtik_amd.modeling.transfer_learning.distributed import fit_distributed
            return fit_distributed(self, dataset, dict(
                epochs=epochs, batch_size=batch_size, lr=lr, eval_dataset=eval_dataset, weight_decay=weight_decay,
                checkpoint_dir=checkpoint_dir, seed=seed, max_steps=max_steps, log_every=log_every,
                warmup_steps=warmup_steps), nnodes, nproc_per_node, hosts, hostfile, shared_dir, launcher)
        import torch.distributed as dist
        from cloudtik_amd.train.trainer import Trainer
        torch.manual_seed(seed)
        if isinstance(dataset, HuggingFaceTextClassificationDataset):
            eval_dataset = eval_dataset if eval_dataset is not None else dataset.validation_subset
            self.classes = self.classes or dataset.class_names
            dataset = dataset.train_subset
        sampler = None
        if dist.is_initialized() and dist.get_world_size() > 1:
            sampler = torch.utils.data.DistributedSampler(dataset, shuffle=True, seed=seed, drop_last=True)
        loader = DataLoader(dataset, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                            drop_last=True, collate_fn=_collate)
        ev = DataLoader(eval_dataset, batch_size=batch_size, collate_fn=_collate) if eval_dataset is not None else None
        sched = None
        if warmup_steps:
            from cloudtik_amd.train.lr_scheduler import LinearWarmupPolyDecayScheduler
            total = max_steps or epochs * max(1, len(loader))
            sched = lambda opt: LinearWarmupPolyDecayScheduler(opt, 0, warmup_steps, total)  # noqa: E731
        no_decay = lambda n: n.endswith("bias") or "ln" in n.split(".")[-1]  # noqa: E731
        tr = Trainer(self.model, optimizer="adamw", lr=lr, weight_decay=weight_decay, train_loader=loader,
                     eval_loader=ev, step_fn=self._step, epochs=epochs, max_steps=max_steps,
                     checkpoint_dir=checkpoint_dir, log_every=log_every, no_decay=no_decay, lr_scheduler=sched)
        try:
            self.history = tr.fit()
        finally:
            tr.close()
        return self.history

    @torch.no_grad()
    def evaluate(self, dataset, batch_size: int = 64) -> Dict[str, float]:
        if isinstance(dataset, HuggingFaceTextClassificationDataset):
            dataset = dataset.validation_subset or dataset.test_subset
        self.model.eval()
        n, correct, loss = 0, 0.0, 0.0
        for b in DataLoader(dataset, batch_size=batch_size, collate_fn=_collate):
            b = {k: v.to(self.device) for k, v in b.items()}
            l, m = self._step(self.model, b)
            k = len(b["label"])
            correct += float(m["accuracy"]) * k
            loss += float(l) * k
            n += k
        self.model.train()
        return {"accuracy": correct / max(n, 1), "loss": loss / max(n, 1)}

    @torch.no_grad()
    def predict(self, inputs, return_raw: bool = False, max_length: int = 128):
        """Class ids (or the raw logits) for a list of strings (needs a tokenizer) or a dict of
        tokenized tensors."""
        if isinstance(inputs, (list, tuple)) and inputs and isinstance(inputs[0], str):
            if self.tokenizer is None:
                raise ValueError("this model has no tokenizer: pass tokenized inputs")
            inputs = self.tokenizer(list(inputs), padding="max_length", truncation=True,
                                    max_length=min(max_length, self.cfg.max_position_embeddings), return_tensors="pt")
        def dev(k):
            v = inputs.get(k)
            return None if v is None else torch.as_tensor(v).to(self.device)

        self.model.eval()
        logits = self.model(dev("input_ids"), dev("attention_mask"), dev("token_type_ids"))
        self.model.train()
        return logits.float() if return_raw else logits.argmax(-1)

    def to_hf(self):
        """A ``transformers.BertForSequenceClassification`` holding the current weights (fp32)."""
        t = _transformers()
        id2label = {i: c for i, c in enumerate(self.classes)} if self.classes else None
        hf = t.BertForSequenceClassification(hf_config_from_bert(self.cfg, self.num_classes, id2label))
        missing, unexpected = hf.load_state_dict(to_hf_state(self.model), strict=False)
        if [k for k in missing if "position_ids" not in k] or [k for k in unexpected if "position_ids" not in k]:
            raise RuntimeError(f"HF export mismatch: missing {missing}, unexpected {unexpected}")
        return hf

    def export(self, output_dir: str) -> str:
        """Standard HF checkpoint (config.json + model.safetensors [+ tokenizer files])."""
        os.makedirs(output_dir, exist_ok=True)
        self.to_hf().save_pretrained(output_dir, safe_serialization=True)
        if self.tokenizer is not None:
            self.tokenizer.save_pretrained(output_dir)
        with open(os.path.join(output_dir, "model_config.json"), "w") as f:
            json.dump({"use_case": self.use_case, "hub": "hugging_face", "model_name": self.model_name,
                       "num_classes": self.num_classes, "classes": self.classes}, f)
        return output_dir

    @classmethod
    def load(cls, output_dir: str, device=None) -> "HuggingFaceTextClassificationModel":
        with open(os.path.join(output_dir, "model_config.json")) as f:
            meta = json.load(f)
        return cls(output_dir, meta["num_classes"], device=device, classes=meta.get("classes"))


def _collate(rows):
    out = {}
    for k in rows[0]:
        v = [r[k] for r in rows]
        out[k] = torch.stack([torch.as_tensor(x) for x in v])
    return out


# ------------------------------------------------------------------ dataset
class _Rows(Dataset):
    def __init__(self, table, columns):
        self.table, self.columns = table, columns

    def __len__(self):
        return len(self.table)

    def __getitem__(self, i):
        r = self.table[int(i)]
        return {c: torch.as_tensor(r[c]) for c in self.columns}


class HuggingFaceTextClassificationDataset:
    """A ``datasets`` text-classification dataset (reference hugging_face/
    text_classification_dataset.py + common/pytorch/hugging_face/dataset.py).

    ``dataset_dir``: a directory written by ``Dataset(Dict).save_to_disk``, or one holding csv /
    json / jsonl / parquet files (a ``train*`` / ``validation*`` / ``test*`` file name picks the
    split); ``dataset_name``: a dataset already in the local HF cache (no download).
    """

    def __init__(self, dataset_dir: str, dataset_name: Optional[str] = None, split: Sequence[str] = ("train",),
                 text_column: Optional[str] = None, label_column: str = "label", shuffle_files: bool = True,
                 num_workers: int = 0, cache_dir: Optional[str] = None):
        import datasets as hfds
        self.dataset_dir, self.dataset_name = dataset_dir, dataset_name
        self.label_column, self.num_workers = label_column, num_workers
        dd = self._load(hfds, dataset_dir, dataset_name, cache_dir)
        self.splits = dd
        wanted = [s for s in split if s in dd] or list(dd)
        self._dataset = hfds.concatenate_datasets([dd[s] for s in wanted]) if len(wanted) > 1 else dd[wanted[0]]
        cols = self._dataset.column_names
        self.text_column = text_column or next((c for c in ("text", "sentence", "review", "content") if c in cols),
                                               next(c for c in cols if c != label_column))
        feat = self._dataset.features.get(label_column)
        if getattr(feat, "names", None):
            self._class_names = list(feat.names)
        else:
            labels = sorted({str(v) for v in self._dataset[label_column]})
            self._class_names = labels
            mapping = {c: i for i, c in enumerate(labels)}
            self._dataset = self._dataset.map(lambda r: {label_column: mapping[str(r[label_column])]})
        self._train = self._val = self._test = None
        self._preprocessed = False
        self._batch_size = 32
        if shuffle_files:
            self._dataset = self._dataset.shuffle(seed=0)

    @staticmethod
    def _load(hfds, dataset_dir, dataset_name, cache_dir):
        if dataset_dir and os.path.isdir(dataset_dir) and (
                os.path.exists(os.path.join(dataset_dir, "dataset_dict.json"))
                or os.path.exists(os.path.join(dataset_dir, "dataset_info.json"))):
            d = hfds.load_from_disk(dataset_dir)
            return d if isinstance(d, hfds.DatasetDict) else hfds.DatasetDict({"train": d})
        if dataset_dir and os.path.isdir(dataset_dir):
            files: Dict[str, List[str]] = {}
            kinds = {".csv": "csv", ".json": "json", ".jsonl": "json", ".parquet": "parquet"}
            kind = None
            for f in sorted(os.listdir(dataset_dir)):
                ext = os.path.splitext(f)[1].lower()
                if ext not in kinds:
                    continue
                kind = kinds[ext]
                sp = next((s for s in ("train", "validation", "test") if f.lower().startswith(s)), "train")
                files.setdefault(sp, []).append(os.path.join(dataset_dir, f))
            if files:
                return hfds.load_dataset(kind, data_files=files, cache_dir=cache_dir)
        if dataset_name:
            return hfds.load_dataset(dataset_name, cache_dir=cache_dir or dataset_dir, download_mode="reuse_cache_if_exists")
        raise ValueError(f"no dataset found in {dataset_dir!r}")

    # ------------------------------------------------------------------ reference API
    @property
    def dataset(self):
        return self._dataset

    @property
    def class_names(self) -> List[str]:
        return list(self._class_names)

    @property
    def info(self) -> Dict[str, Any]:
        return {"name": self.dataset_name or os.path.basename(str(self.dataset_dir)), "size": len(self._dataset),
                "classes": self.class_names, "text_column": self.text_column}

    def __len__(self):
        return len(self._dataset)

    def preprocess(self, tokenizer=None, batch_size: int = 32, max_length: int = 128, padding: str = "max_length",
                   truncation: bool = True):
        """Tokenize the text column.  ``tokenizer``: an HF tokenizer object, a local tokenizer
        directory / model name, or None (the hash tokenizer of datasets.py)."""
        self._batch_size = batch_size
        if tokenizer is None:
            from .datasets import HashTokenizer
            ht = HashTokenizer(max_length=max_length)

            def tok(batch):
                ids, mask = ht(batch[self.text_column])
                return {"input_ids": ids.tolist(), "attention_mask": mask.tolist()}
        else:
            if isinstance(tokenizer, str):
                tokenizer = _transformers().AutoTokenizer.from_pretrained(tokenizer, local_files_only=True)

            def tok(batch):
                enc = tokenizer(batch[self.text_column], padding=padding, truncation=truncation, max_length=max_length)
                return {k: enc[k] for k in ("input_ids", "attention_mask", "token_type_ids") if k in enc}
        self._dataset = self._dataset.map(tok, batched=True)
        self._preprocessed = True
        self._train = self._val = self._test = None
        return self

    def shuffle_split(self, train_pct: float = 0.75, val_pct: float = 0.25, test_pct: float = 0.0,
                      shuffle_files: bool = True, seed: Optional[int] = None):
        if abs(train_pct + val_pct + test_pct - 1.0) > 1e-6:
            raise ValueError("percentages must sum to 1")
        n = len(self._dataset)
        idx = np.random.default_rng(seed).permutation(n) if shuffle_files else np.arange(n)
        a, b = int(n * train_pct), int(n * (train_pct + val_pct))
        self._split_idx = (idx[:a], idx[a:b], idx[b:])
        self._train = self._val = self._test = None
        return self

    def _subset(self, which: int):
        if not self._preprocessed:
            raise RuntimeError("call preprocess() first")
        if not hasattr(self, "_split_idx"):
            self.shuffle_split()
        idx = self._split_idx[which]
        if len(idx) == 0:
            return None
        cols = [c for c in ("input_ids", "attention_mask", "token_type_ids") if c in self._dataset.column_names]
        return _Rows(self._dataset.select(idx.tolist()), cols + [self.label_column]) if self.label_column == "label" \
            else _RenamedRows(self._dataset.select(idx.tolist()), cols, self.label_column)

    @property
    def train_subset(self):
        return self._subset(0)

    @property
    def validation_subset(self):
        return self._subset(1)

    @property
    def test_subset(self):
        return self._subset(2)

    def _loader(self, sub, shuffle):
        return None if sub is None else DataLoader(sub, batch_size=self._batch_size, shuffle=shuffle,
                                                   num_workers=self.num_workers, collate_fn=_collate)

    @property
    def train_loader(self):
        return self._loader(self.train_subset, True)

    @property
    def validation_loader(self):
        return self._loader(self.validation_subset, False)

    @property
    def test_loader(self):
        return self._loader(self.test_subset, False)


class _RenamedRows(_Rows):
    def __init__(self, table, columns, label_column):
        super().__init__(table, columns + [label_column])
        self.label_column = label_column

    def __getitem__(self, i):
        r = super().__getitem__(i)
        r["label"] = r.pop(self.label_column)
        return r
