"""Image-classification transfer learning (reference modeling/transfer_learning/
image_classification/pytorch/image_classification_model.py:247-330 and
common/pytorch/trainer.py:87-240: torchvision backbone, new classifier head, optional frozen
backbone, DDP training, checkpoint + export).

The backbone is the framework's own bf16 channels-last ResNet (MIOpen convolutions, fused
BN+ReLU, HIP fused optimizers); training goes through ``train.Trainer`` (flat parameter
space, bucketed RCCL all-reduce when launched with several ranks).  Pretrained weights come
from a local safetensors / torch file (no hub downloads here).
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset

from cloudtik_amd.models.resnet import ResNet

BACKBONES = {"resnet50": (3, 4, 6, 3), "resnet101": (3, 4, 23, 3), "resnet152": (3, 8, 36, 3),
             "resnet_tiny": (1, 1, 1, 1)}


def _default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def load_state_file(path: str) -> Dict[str, torch.Tensor]:
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return sd.get("state_dict", sd) if isinstance(sd, dict) else sd


def load_pretrained(model: nn.Module, path: str, skip_prefixes=("fc.",)) -> List[str]:
    """Copy matching tensors (name and shape) into ``model``; returns the names loaded."""
    sd = load_state_file(path)
    own = model.state_dict()
    loaded = []
    for k, v in sd.items():
        if k.startswith(tuple(skip_prefixes)) or k not in own or own[k].shape != v.shape:
            continue
        own[k].copy_(v.to(own[k].dtype))
        loaded.append(k)
    return loaded


class ImageClassificationModel:
    use_case = "image_classification"

    def __init__(self, model_name: str = "resnet50", num_classes: int = 2, pretrained_path: Optional[str] = None,
                 freeze_backbone: bool = True, device=None, dtype: Optional[torch.dtype] = None,
                 classes: Optional[List[str]] = None):
        if model_name not in BACKBONES:
            raise ValueError(f"unsupported image model {model_name!r}; choose from {sorted(BACKBONES)}")
        self.model_name, self.num_classes = model_name, num_classes
        self.device = torch.device(device) if device else _default_device()
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.classes = classes
        net = ResNet(BACKBONES[model_name], 1000, device=self.device, dtype=self.dtype)
        if pretrained_path:
            load_pretrained(net, pretrained_path)
        in_f = net.fc.in_features
        net.fc = nn.Linear(in_f, num_classes, device=self.device, dtype=self.dtype)
        self.freeze_backbone = freeze_backbone
        if freeze_backbone:
            for n, p in net.named_parameters():
                p.requires_grad_(n.startswith("fc."))
        self.model = net
        self.history: List[Dict[str, float]] = []

    # ---------------------------------------------------------------- training
    def _step(self, model, batch):
        x, y = batch
        x = x.to(self.dtype)
        if self.device.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
        if self.freeze_backbone:
            model.eval()                       # frozen BN statistics
        out = model(x)
        loss = F.cross_entropy(out.float(), y)
        return loss, {"loss": loss.detach(), "accuracy": (out.argmax(-1) == y).float().mean()}

    def _loader(self, ds: Dataset, batch_size: int, shuffle: bool, seed: int = 0):
        import torch.distributed as dist
        sampler = None
        if dist.is_initialized() and dist.get_world_size() > 1:
            sampler = torch.utils.data.DistributedSampler(ds, shuffle=shuffle, seed=seed, drop_last=True)
        return DataLoader(ds, batch_size=batch_size, shuffle=shuffle and sampler is None, sampler=sampler,
                          drop_last=shuffle, num_workers=0, pin_memory=self.device.type == "cuda")

    def train(self, dataset: Dataset, epochs: int = 1, batch_size: int = 32, lr: float = 1e-3,
              eval_dataset: Optional[Dataset] = None, optimizer: str = "adamw", weight_decay: float = 0.0,
              checkpoint_dir: Optional[str] = None, seed: int = 0, max_steps: Optional[int] = None,
              log_every: int = 50, distributed: bool = False, nnodes: int = 1, nproc_per_node: int = 1,
              hosts: Optional[str] = None, hostfile: Optional[str] = None, shared_dir: Optional[str] = None,
              launcher: Optional[str] = None) -> List[Dict[str, float]]:
        """Fine-tune; ``distributed=True`` launches ``nnodes`` x ``nproc_per_node`` ranks through
        cloudtik-run from here (modeling/transfer_learning/distributed.py)."""
        if distributed:
            from cloudtik_amd.modeling.transfer_learning.distributed import fit_distributed
            return fit_distributed(self, dataset, dict(
                epochs=epochs, batch_size=batch_size, lr=lr, eval_dataset=eval_dataset, optimizer=optimizer,
                weight_decay=weight_decay, checkpoint_dir=checkpoint_dir, seed=seed, max_steps=max_steps,
                log_every=log_every), nnodes, nproc_per_node, hosts, hostfile, shared_dir, launcher)
        from cloudtik_amd.train.trainer import Trainer
        self.classes = self.classes or getattr(dataset, "classes", None)
        tr = Trainer(self.model, optimizer=optimizer, lr=lr, weight_decay=weight_decay,
                     train_loader=self._loader(dataset, batch_size, True, seed),
                     eval_loader=self._loader(eval_dataset, batch_size, False) if eval_dataset is not None else None,
                     step_fn=self._step, epochs=epochs, max_steps=max_steps, checkpoint_dir=checkpoint_dir,
                     log_every=log_every)
        try:
            self.history = tr.fit()
        finally:
            tr.close()
        return self.history

    @torch.no_grad()
    def evaluate(self, dataset: Dataset, batch_size: int = 64) -> Dict[str, float]:
        self.model.eval()
        n, correct, loss = 0, 0, 0.0
        for x, y in DataLoader(dataset, batch_size=batch_size):
            x, y = x.to(self.device), y.to(self.device)
            l, m = self._step(self.model, (x, y))
            correct += float(m["accuracy"]) * len(y)
            loss += float(l) * len(y)
            n += len(y)
        return {"accuracy": correct / max(n, 1), "loss": loss / max(n, 1)}

    @torch.no_grad()
    def predict(self, images: torch.Tensor) -> torch.Tensor:
        self.model.eval()
        x = images.to(self.device, self.dtype)
        if self.device.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
        return torch.softmax(self.model(x).float(), -1)

    # ---------------------------------------------------------------- persistence
    def export(self, output_dir: str) -> str:
        from safetensors.torch import save_file
        os.makedirs(output_dir, exist_ok=True)
        path = os.path.join(output_dir, "model.safetensors")
        save_file({k: v.detach().contiguous().cpu() for k, v in self.model.state_dict().items()}, path)
        with open(os.path.join(output_dir, "model_config.json"), "w") as f:
            json.dump({"use_case": self.use_case, "model_name": self.model_name, "num_classes": self.num_classes,
                       "classes": self.classes}, f)
        return path

    @classmethod
    def load(cls, output_dir: str, device=None) -> "ImageClassificationModel":
        with open(os.path.join(output_dir, "model_config.json")) as f:
            cfg = json.load(f)
        m = cls(cfg["model_name"], cfg["num_classes"], freeze_backbone=False, device=device, classes=cfg["classes"])
        sd = load_state_file(os.path.join(output_dir, "model.safetensors"))
        m.model.load_state_dict({k: v.to(m.dtype) if v.is_floating_point() else v for k, v in sd.items()})
        return m
