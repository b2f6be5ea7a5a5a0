"""TransNetV2 shot-boundary detection (inference).

Reference workload: the quickstart TransNetV2 inference (applications/ai/quickstart,
SURVEY.md §2.12).  Same topology with random-init weights: 100-frame windows of 48x27 RGB
frames -> 3 stacked SDDCNN blocks (each 2 DDCNN cells of four dilated (1, 2, 4, 8)
factorised 3-D convolutions: 3x3 spatial then 3-tap temporal) with 2x2 spatial pooling ->
frame-similarity features (cosine similarity of pooled block features within +-50 frames)
and RGB colour-histogram similarities -> per-frame dense layer -> two heads
(single-frame and all-frame transition logits).

MI355X mapping: frames are processed as NDHWC bf16 (``channels_last_3d``) so the 3-D
convolutions map onto MIOpen's channels-last kernels; the frame-similarity and histogram
windows are single batched GEMMs + one gather (no per-frame loops).
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class DilatedDCNN(nn.Module):
    """Four parallel factorised 3-D convs with temporal dilations 1, 2, 4, 8, concatenated."""

    def __init__(self, cin: int, filters: int, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.spatial = nn.ModuleList([nn.Conv3d(cin, 2 * filters, (1, 3, 3), padding=(0, 1, 1), bias=False, **kw)
                                      for _ in range(4)])
        self.temporal = nn.ModuleList([nn.Conv3d(2 * filters, filters, (3, 1, 1), padding=(d, 0, 0),
                                                 dilation=(d, 1, 1), bias=False, **kw) for d in (1, 2, 4, 8)])
        self.bn = nn.BatchNorm3d(4 * filters, eps=1e-3, **kw)

    def forward(self, x):
        y = torch.cat([t(s(x)) for s, t in zip(self.spatial, self.temporal)], 1)
        return F.relu(self.bn(y))


class StackedDDCNN(nn.Module):
    def __init__(self, cin: int, filters: int, cells: int = 2, device=None, dtype=None):
        super().__init__()
        layers, c = [], cin
        for _ in range(cells):
            layers.append(DilatedDCNN(c, filters, device, dtype))
            c = 4 * filters
        self.cells = nn.ModuleList(layers)
        self.out_channels = c

    def forward(self, x):
        shortcut = None
        for i, cell in enumerate(self.cells):
            x = cell(x)
            if i == 0:
                shortcut = x
        x = x + shortcut                       # residual over the block
        return F.avg_pool3d(x, (1, 2, 2))


class FrameSimilarity(nn.Module):
    """Cosine similarities between each frame's pooled features and its +-lookup neighbours."""

    def __init__(self, in_features: int, similarity_dim: int = 128, lookup: int = 101, out: int = 128,
                 device=None, dtype=None):
        super().__init__()
        self.proj = nn.Linear(in_features, similarity_dim, bias=False, device=device, dtype=dtype)
        self.fc = nn.Linear(lookup, out, device=device, dtype=dtype)
        self.lookup = lookup

    def forward(self, feats):
        # feats: list of [B, C_i, T, H_i, W_i] block outputs
        x = torch.cat([f.mean(dim=(3, 4)) for f in feats], 1).transpose(1, 2)        # [B, T, sum C]
        x = F.normalize(self.proj(x).float(), dim=-1)
        sim = torch.bmm(x, x.transpose(1, 2))                                         # [B, T, T]
        B, T, _ = sim.shape
        half = self.lookup // 2
        sim = F.pad(sim, (half, half))
        idx = torch.arange(T, device=sim.device)[:, None] + torch.arange(self.lookup, device=sim.device)[None]
        win = sim.gather(2, idx.unsqueeze(0).expand(B, T, self.lookup))               # [B, T, lookup]
        return F.relu(self.fc(win.to(self.fc.weight.dtype)))


class ColorHistograms(nn.Module):
    """512-bin RGB histograms per frame -> windowed histogram similarities -> dense."""

    def __init__(self, lookup: int = 101, out: int = 128, device=None, dtype=None):
        super().__init__()
        self.fc = nn.Linear(lookup, out, device=device, dtype=dtype)
        self.lookup = lookup

    def forward(self, frames_u8):
        # frames [B, T, H, W, 3] uint8 -> 8x8x8 bins
        B, T = frames_u8.shape[:2]
        q = (frames_u8.long() >> 5)
        bins = (q[..., 0] << 6) + (q[..., 1] << 3) + q[..., 2]                        # [B, T, H, W]
        flat = bins.reshape(B * T, -1)
        hist = torch.zeros(B * T, 512, device=frames_u8.device).scatter_add_(
            1, flat, torch.ones_like(flat, dtype=torch.float32))
        hist = F.normalize(hist.view(B, T, 512), dim=-1)
        sim = torch.bmm(hist, hist.transpose(1, 2))
        half = self.lookup // 2
        sim = F.pad(sim, (half, half))
        idx = torch.arange(T, device=sim.device)[:, None] + torch.arange(self.lookup, device=sim.device)[None]
        win = sim.gather(2, idx.unsqueeze(0).expand(B, T, self.lookup))
        return F.relu(self.fc(win.to(self.fc.weight.dtype)))


class TransNetV2(nn.Module):
    def __init__(self, filters: int = 16, layers: int = 3, dense: int = 1024, device=None, dtype=torch.bfloat16,
                 input_size: Tuple[int, int] = (27, 48)):
        super().__init__()
        blocks, c = [], 3
        for i in range(layers):
            blk = StackedDDCNN(c, filters * 2 ** i, device=device, dtype=dtype)
            blocks.append(blk)
            c = blk.out_channels
        self.blocks = nn.ModuleList(blocks)
        h, w = input_size
        for _ in range(layers):
            h, w = h // 2, w // 2
        self.sim = FrameSimilarity(sum(b.out_channels for b in self.blocks), device=device, dtype=dtype)
        self.hist = ColorHistograms(device=device, dtype=dtype)
        self.fc1 = nn.Linear(c * h * w + 128 + 128, dense, device=device, dtype=dtype)
        self.cls_one = nn.Linear(dense, 1, device=device, dtype=dtype)
        self.cls_all = nn.Linear(dense, 1, device=device, dtype=dtype)
        self.dtype = dtype
        if device is not None and torch.device(device).type == "cuda":
            self.to(memory_format=torch.channels_last_3d)

    def forward(self, frames_u8: torch.Tensor):
        """frames [B, T, 27, 48, 3] uint8 -> (single-frame logits [B, T], all-frame logits [B, T])."""
        x = frames_u8.permute(0, 4, 1, 2, 3).to(self.dtype) / 255.0                   # [B, 3, T, H, W]
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last_3d)
        feats = []
        for blk in self.blocks:
            x = blk(x)
            feats.append(x)
        B, C, T, H, W = x.shape
        flat = x.permute(0, 2, 3, 4, 1).reshape(B, T, H * W * C)
        h = torch.cat([flat, self.sim(feats), self.hist(frames_u8)], -1)
        h = F.relu(self.fc1(h))
        return self.cls_one(h).squeeze(-1), self.cls_all(h).squeeze(-1)

    @torch.no_grad()
    def predict_transitions(self, frames_u8: torch.Tensor, threshold: float = 0.5) -> torch.Tensor:
        one, _ = self(frames_u8)
        return torch.sigmoid(one.float()) > threshold
