"""Text-classification transfer learning (reference modeling/transfer_learning/
text_classification/pytorch/text_classification_model.py: HF BERT + classifier head).

Encoder = the framework's BERT (HIP fused attention / LayerNorm / bias-GELU kernels), head
= dropout + linear over the pooled [CLS] output.  Pretrained encoder weights load from a
local safetensors / torch file with matching parameter names.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset

from cloudtik_amd.models.bert import BertConfig, BertModel

from .image_classification import _default_device, load_pretrained, load_state_file

ENCODERS = {"bert-large-uncased": BertConfig.large, "bert-base-uncased": BertConfig.base, "bert-tiny": BertConfig.tiny}


class BertClassifier(nn.Module):
    def __init__(self, cfg: BertConfig, num_classes: int, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.bert = BertModel(cfg, device=device, dtype=dtype)
        self.dropout = cfg.hidden_dropout_prob
        self.classifier = nn.Linear(cfg.hidden_size, num_classes, device=device, dtype=dtype)

    def forward(self, input_ids, attention_mask=None, token_type_ids=None):
        _, pooled = self.bert(input_ids, token_type_ids, attention_mask)
        return self.classifier(F.dropout(pooled, self.dropout, self.training))


class TextClassificationModel:
    use_case = "text_classification"

    def __init__(self, model_name: str = "bert-base-uncased", num_classes: int = 2,
                 pretrained_path: Optional[str] = None, freeze_encoder: bool = False, device=None,
                 dtype: Optional[torch.dtype] = None, classes: Optional[List[str]] = None, **config_overrides):
        if model_name not in ENCODERS:
            raise ValueError(f"unsupported text model {model_name!r}; choose from {sorted(ENCODERS)}")
        self.model_name, self.num_classes, self.classes = model_name, num_classes, classes
        self.device = torch.device(device) if device else _default_device()
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.cfg = ENCODERS[model_name](**config_overrides)
        self.model = BertClassifier(self.cfg, num_classes, device=self.device, dtype=self.dtype)
        if pretrained_path:
            load_pretrained(self.model.bert, pretrained_path, skip_prefixes=("cls.", "classifier."))
        if freeze_encoder:
            for p in self.model.bert.parameters():
                p.requires_grad_(False)
        self.history: List[Dict[str, float]] = []

    @staticmethod
    def _step(model, batch):
        out = model(batch["input_ids"], batch["attention_mask"])
        y = batch["label"]
        loss = F.cross_entropy(out.float(), y)
        return loss, {"loss": loss.detach(), "accuracy": (out.argmax(-1) == y).float().mean()}

    def train(self, dataset: Dataset, epochs: int = 1, batch_size: int = 32, lr: float = 2e-5,
              eval_dataset: Optional[Dataset] = None, optimizer: str = "adamw", weight_decay: float = 0.01,
              checkpoint_dir: Optional[str] = None, seed: int = 0, max_steps: Optional[int] = None,
              log_every: int = 50, distributed: bool = False, nnodes: int = 1, nproc_per_node: int = 1,
              hosts: Optional[str] = None, hostfile: Optional[str] = None, shared_dir: Optional[str] = None,
              launcher: Optional[str] = None) -> List[Dict[str, float]]:
        if distributed:
            from cloudtik_amd.modeling.transfer_learning.distributed import fit_distributed
            return fit_distributed(self, dataset, dict(
                epochs=epochs, batch_size=batch_size, lr=lr, eval_dataset=eval_dataset, optimizer=optimizer,
                weight_decay=weight_decay, checkpoint_dir=checkpoint_dir, seed=seed, max_steps=max_steps,
                log_every=log_every), nnodes, nproc_per_node, hosts, hostfile, shared_dir, launcher)
        import torch.distributed as dist
        from cloudtik_amd.train.trainer import Trainer
        self.classes = self.classes or getattr(dataset, "classes", None)
        sampler = None
        if dist.is_initialized() and dist.get_world_size() > 1:
            sampler = torch.utils.data.DistributedSampler(dataset, shuffle=True, seed=seed, drop_last=True)
        loader = DataLoader(dataset, batch_size=batch_size, shuffle=sampler is None, sampler=sampler, drop_last=True)
        ev = DataLoader(eval_dataset, batch_size=batch_size) if eval_dataset is not None else None
        no_decay = lambda n: n.endswith("bias") or "ln_" in n or "layer_norm" in n or "norm" in n
        tr = Trainer(self.model, optimizer=optimizer, lr=lr, weight_decay=weight_decay, train_loader=loader,
                     eval_loader=ev, step_fn=self._step, epochs=epochs, max_steps=max_steps,
                     checkpoint_dir=checkpoint_dir, log_every=log_every, no_decay=no_decay)
        try:
            self.history = tr.fit()
        finally:
            tr.close()
        return self.history

    @torch.no_grad()
    def evaluate(self, dataset: Dataset, batch_size: int = 64) -> Dict[str, float]:
        self.model.eval()
        n, correct = 0, 0.0
        for b in DataLoader(dataset, batch_size=batch_size):
            b = {k: v.to(self.device) for k, v in b.items()}
            _, m = self._step(self.model, b)
            correct += float(m["accuracy"]) * len(b["label"])
            n += len(b["label"])
        self.model.train()
        return {"accuracy": correct / max(n, 1)}

    @torch.no_grad()
    def predict(self, input_ids: torch.Tensor, attention_mask: torch.Tensor) -> torch.Tensor:
        self.model.eval()
        return torch.softmax(self.model(input_ids.to(self.device), attention_mask.to(self.device)).float(), -1)

    def export(self, output_dir: str) -> str:
        from safetensors.torch import save_file
        os.makedirs(output_dir, exist_ok=True)
        path = os.path.join(output_dir, "model.safetensors")
        save_file({k: v.detach().contiguous().cpu() for k, v in self.model.state_dict().items()}, path)
        with open(os.path.join(output_dir, "model_config.json"), "w") as f:
            json.dump({"use_case": self.use_case, "model_name": self.model_name, "num_classes": self.num_classes,
                       "classes": self.classes, "bert": self.cfg.to_dict()}, f)
        return path

    @classmethod
    def load(cls, output_dir: str, device=None) -> "TextClassificationModel":
        with open(os.path.join(output_dir, "model_config.json")) as f:
            cfg = json.load(f)
        overrides = {k: v for k, v in cfg["bert"].items()}
        m = cls(cfg["model_name"], cfg["num_classes"], device=device, classes=cfg["classes"], **overrides)
        sd = load_state_file(os.path.join(output_dir, "model.safetensors"))
        m.model.load_state_dict({k: v.to(m.dtype) if v.is_floating_point() else v for k, v in sd.items()})
        return m
