"""Image anomaly detection by transfer learning (reference modeling/transfer_learning/
image_anomaly_detection/pytorch/: image_anomaly_detection_model.py:52-620, cutpaste/,
simsiam/).

Only "good" images are needed for training (MVTec-style folders ``train/good``,
``test/good``, ``test/<defect>``):

1. a backbone (the framework's bf16 channels-last ResNet; optional local pretrained
   weights) turns each image into a pooled feature vector of one stage (``layer3`` by
   default: mid-level texture features transfer best to defect detection);
2. optionally the backbone is first adapted to the domain with a self-supervised task on
   the good images: **CutPaste** (classify normal vs. an image with a patch cut and pasted
   elsewhere -- and the thin "scar" variant) or **SimSiam** (two augmented views, predictor
   MLP, negative cosine similarity with stop-gradient);
3. PCA of the good features keeps the components explaining ``variance_threshold`` of the
   variance; the anomaly score of an image is its feature's reconstruction error outside
   that subspace.  ``evaluate`` reports AUROC over good vs. defective test images.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .image_classification import BACKBONES, _default_device, load_pretrained

IMG_EXT = (".png", ".jpg", ".jpeg", ".bmp")


# ------------------------------------------------------------------------------------ data
class AnomalyImageFolder(torch.utils.data.Dataset):
    """``root/<split>/good`` -> label 0, ``root/<split>/<any other dir>`` -> label 1."""

    def __init__(self, root: str, split: str = "train", image_size: int = 224):
        from PIL import Image  # noqa: F401  (fail early if PIL is missing)
        self.items: List[Tuple[str, int]] = []
        base = os.path.join(root, split)
        for d in sorted(os.listdir(base)):
            full = os.path.join(base, d)
            if not os.path.isdir(full):
                continue
            for f in sorted(os.listdir(full)):
                if f.lower().endswith(IMG_EXT):
                    self.items.append((os.path.join(full, f), 0 if d == "good" else 1))
        self.image_size = image_size

    def __len__(self):
        return len(self.items)

    def __getitem__(self, i):
        from PIL import Image
        path, label = self.items[i]
        img = Image.open(path).convert("RGB").resize((self.image_size, self.image_size))
        x = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0).permute(2, 0, 1)
        mean = torch.tensor([0.485, 0.456, 0.406]).view(3, 1, 1)
        std = torch.tensor([0.229, 0.224, 0.225]).view(3, 1, 1)
        return (x - mean) / std, label


# ------------------------------------------------------------------------------ augmentations
def cutpaste(x: torch.Tensor, generator: torch.Generator, scar: bool = False) -> torch.Tensor:
    """One CutPaste (or CutPaste-scar) augmentation of a [C, H, W] image: a random patch
    (area 2-15 % with aspect 0.3-3.3; scar: 2-16 x 10-25 px thin strip) is cut, colour-jittered
    and pasted at another random location."""
    C, H, W = x.shape
    r = lambda lo, hi: float(lo + (hi - lo) * torch.rand((), generator=generator))  # noqa: E731
    if scar:
        pw, ph = max(2, int(r(2, 16) * W / 224)), max(4, int(r(10, 25) * H / 224))
    else:
        area = r(0.02, 0.15) * H * W
        aspect = math.exp(r(math.log(0.3), math.log(1 / 0.3)))
        pw = max(2, min(W - 1, int(math.sqrt(area * aspect))))
        ph = max(2, min(H - 1, int(math.sqrt(area / aspect))))
    sx, sy = int(r(0, W - pw)), int(r(0, H - ph))
    dx, dy = int(r(0, W - pw)), int(r(0, H - ph))
    patch = x[:, sy:sy + ph, sx:sx + pw].clone()
    patch = patch * r(0.9, 1.1) + r(-0.1, 0.1)            # brightness / contrast jitter
    out = x.clone()
    out[:, dy:dy + ph, dx:dx + pw] = patch
    return out


def simsiam_views(x: torch.Tensor, generator: torch.Generator) -> torch.Tensor:
    """A light augmentation for SimSiam views: random resized crop + flip + noise."""
    C, H, W = x.shape
    s = float(0.6 + 0.4 * torch.rand((), generator=generator))
    ch, cw = max(4, int(H * s)), max(4, int(W * s))
    y0 = int(torch.randint(0, H - ch + 1, (), generator=generator))
    x0 = int(torch.randint(0, W - cw + 1, (), generator=generator))
    v = F.interpolate(x[None, :, y0:y0 + ch, x0:x0 + cw], size=(H, W), mode="bilinear", align_corners=False)[0]
    if torch.rand((), generator=generator) < 0.5:
        v = v.flip(-1)
    return v + 0.05 * torch.randn(v.shape, generator=generator)


# ------------------------------------------------------------------------------------ model
class ImageAnomalyDetectionModel:
    use_case = "image_anomaly_detection"
    LAYERS = ("layer1", "layer2", "layer3", "layer4")

    def __init__(self, model_name: str = "resnet50", layer_name: str = "layer3", pooling: str = "avg",
                 pretrained_path: Optional[str] = None, device=None, dtype: Optional[torch.dtype] = None):
        from cloudtik_amd.models.resnet import ResNet
        if model_name not in BACKBONES:
            raise ValueError(f"unsupported backbone {model_name!r}; choose from {sorted(BACKBONES)}")
        if layer_name not in self.LAYERS or pooling not in ("avg", "max"):
            raise ValueError("layer_name must be layer1..layer4 and pooling avg|max")
        self.device = torch.device(device) if device else _default_device()
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        self.net = ResNet(BACKBONES[model_name], 1000, device=self.device, dtype=self.dtype)
        if pretrained_path:
            load_pretrained(self.net, pretrained_path)
        self.model_name, self.layer_name, self.pooling = model_name, layer_name, pooling
        self.pca: Optional[Dict[str, torch.Tensor]] = None

    # ---------------------------------------------------------------- features
    def _stage_out(self, x: torch.Tensor) -> torch.Tensor:
        n = self.net
        h = n.stem(x)
        for name in self.LAYERS:
            h = getattr(n, name)(h)
            if name == self.layer_name:
                return h
        return h

    def _pool(self, h: torch.Tensor) -> torch.Tensor:
        return (F.adaptive_avg_pool2d(h, 1) if self.pooling == "avg" else F.adaptive_max_pool2d(h, 1)).flatten(1)

    def _prep(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(self.device, self.dtype)
        return x.contiguous(memory_format=torch.channels_last) if self.device.type == "cuda" else x

    @torch.no_grad()
    def extract_features(self, images) -> torch.Tensor:
        """[N, C] float32 pooled features of ``layer_name`` (images: tensor or iterable of batches)."""
        self.net.eval()
        batches = [images] if isinstance(images, torch.Tensor) else (b[0] if isinstance(b, (list, tuple)) else b
                                                                        for b in images)
        return torch.cat([self._pool(self._stage_out(self._prep(x))).float().cpu() for x in batches])

    # ---------------------------------------------------------------- PCA scoring
    def fit_pca(self, features: torch.Tensor, variance_threshold: float = 0.99) -> Dict[str, torch.Tensor]:
        f = features.double()
        mean = f.mean(0)
        _, s, vt = torch.linalg.svd(f - mean, full_matrices=False)
        var = s ** 2
        k = int(torch.searchsorted(torch.cumsum(var, 0) / var.sum().clamp_min(1e-30),
                                   torch.tensor(variance_threshold, dtype=var.dtype)).item()) + 1
        self.pca = {"mean": mean, "components": vt[:min(k, vt.shape[0])]}
        return self.pca

    def score(self, features: torch.Tensor) -> torch.Tensor:
        """Squared reconstruction error of each feature outside the good-image subspace."""
        if self.pca is None:
            raise RuntimeError("fit_pca() first (train() does it)")
        f = features.double() - self.pca["mean"]
        comp = self.pca["components"]
        recon = (f @ comp.T) @ comp
        return ((f - recon) ** 2).sum(1).float()

    # ---------------------------------------------------------------- training
    def _self_supervised(self, loader, method: str, epochs: int, lr: float, seed: int) -> List[float]:
        g = torch.Generator().manual_seed(seed)
        feat_dim = self._pool(self._stage_out(self._prep(next(iter(loader))[0][:1]))).shape[1]
        kw = dict(device=self.device, dtype=self.dtype)
        if method == "cutpaste":
            head = nn.Sequential(nn.Linear(feat_dim, 128, **kw), nn.ReLU(), nn.Linear(128, 3, **kw))
        else:   # simsiam: projector + predictor
            head = nn.ModuleDict({
                "proj": nn.Sequential(nn.Linear(feat_dim, 128, **kw), nn.ReLU(), nn.Linear(128, 128, **kw)),
                "pred": nn.Sequential(nn.Linear(128, 32, **kw), nn.ReLU(), nn.Linear(32, 128, **kw))})
        params = [p for p in self.net.parameters()] + list(head.parameters())
        opt = torch.optim.SGD(params, lr=lr, momentum=0.9, weight_decay=1e-4)
        losses = []
        self.net.train()
        for _ in range(epochs):
            tot, n = 0.0, 0
            for x, _ in loader:
                if method == "cutpaste":
                    # 3-way: normal / cutpaste / scar (reference cutpaste.py CutPaste3Way)
                    xs = torch.cat([x, torch.stack([cutpaste(i, g) for i in x]),
                                    torch.stack([cutpaste(i, g, scar=True) for i in x])])
                    y = torch.arange(3).repeat_interleave(len(x)).to(self.device)
                    logits = head(self._pool(self._stage_out(self._prep(xs))))
                    loss = F.cross_entropy(logits.float(), y)
                else:
                    v1 = torch.stack([simsiam_views(i, g) for i in x])
                    v2 = torch.stack([simsiam_views(i, g) for i in x])
                    z1 = head["proj"](self._pool(self._stage_out(self._prep(v1))))
                    z2 = head["proj"](self._pool(self._stage_out(self._prep(v2))))
                    p1, p2 = head["pred"](z1), head["pred"](z2)
                    loss = -(F.cosine_similarity(p1.float(), z2.detach().float()).mean() +
                             F.cosine_similarity(p2.float(), z1.detach().float()).mean()) / 2
                opt.zero_grad(set_to_none=True)
                loss.backward()
                opt.step()
                tot += float(loss.detach())
                n += 1
            losses.append(tot / max(1, n))
        self.net.eval()
        return losses

    def train(self, dataset, batch_size: int = 32, method: str = "none", epochs: int = 1, lr: float = 0.01,
              variance_threshold: float = 0.99, seed: int = 0) -> Dict[str, object]:
        """Fit on the good images of ``dataset`` (label 0 rows): optional self-supervised
        adaptation (``cutpaste`` / ``simsiam``), then the PCA of their features."""
        if method not in ("none", "cutpaste", "simsiam"):
            raise ValueError("method must be none, cutpaste or simsiam")
        good = [i for i in range(len(dataset)) if dataset[i][1] == 0] if hasattr(dataset, "__getitem__") else None
        subset = torch.utils.data.Subset(dataset, good) if good is not None else dataset
        loader = torch.utils.data.DataLoader(subset, batch_size=batch_size, shuffle=True,
                                             generator=torch.Generator().manual_seed(seed))
        losses = self._self_supervised(loader, method, epochs, lr, seed) if method != "none" else []
        feats = self.extract_features(torch.utils.data.DataLoader(subset, batch_size=batch_size))
        pca = self.fit_pca(feats, variance_threshold)
        return {"ssl_losses": losses, "pca_components": int(pca["components"].shape[0]),
                "train_images": len(subset)}

    def evaluate(self, dataset, batch_size: int = 32) -> Dict[str, float]:
        from sklearn.metrics import roc_auc_score
        loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size)
        scores = self.score(self.extract_features(loader)).numpy()
        labels = np.array([dataset[i][1] for i in range(len(dataset))])
        out = {"images": int(len(labels)), "defective": int(labels.sum())}
        if 0 < labels.sum() < len(labels):
            out["auroc"] = float(roc_auc_score(labels, scores))
        return out

    # ---------------------------------------------------------------- persistence
    def save(self, output_dir: str):
        import json
        os.makedirs(output_dir, exist_ok=True)
        torch.save({"backbone": self.net.state_dict(), "pca": self.pca}, os.path.join(output_dir, "model.pt"))
        with open(os.path.join(output_dir, "model_config.json"), "w") as f:
            json.dump({"use_case": self.use_case, "model_name": self.model_name, "layer_name": self.layer_name,
                       "pooling": self.pooling}, f)
        return output_dir

    @classmethod
    def load(cls, output_dir: str, device=None):
        import json
        with open(os.path.join(output_dir, "model_config.json")) as f:
            c = json.load(f)
        m = cls(c["model_name"], c["layer_name"], c["pooling"], device=device)
        sd = torch.load(os.path.join(output_dir, "model.pt"), map_location=m.device, weights_only=True)
        m.net.load_state_dict(sd["backbone"])
        m.pca = {k: v.cpu() for k, v in sd["pca"].items()} if sd.get("pca") else None
        return m

    def predict(self, images: torch.Tensor, threshold: Optional[float] = None, return_type: str = "scores"):
        s = self.score(self.extract_features(images))
        if return_type == "scores":
            return s
        if threshold is None:
            raise ValueError("class prediction needs a numeric threshold")
        return (s > threshold).long()
