"""RNN-Transducer speech recognition model (MLPerf RNN-T topology).

Reference workload: the quickstart RNN-T training / inference
(applications/ai/quickstart/bin/rnnt/*, models/language_modeling/pytorch/rnnt: LSTM encoder
with time stacking, LSTM prediction network, joint network, transducer loss, greedy
decoding).

MI355X mapping:
* LSTMs run through MIOpen's fused RNN kernels in fp32 (``run_lstm``: MIOpen has no bf16
  RNN, and the bf16 fallback is a per-time-step kernel loop 4x slower);
* the joint network is one broadcast-add + ReLU over [B, T, U+1, H] followed by one GEMM to
  the vocabulary;
* the transducer loss is the HIP lattice kernel set of ``ops.rnnt_loss`` (log-softmax
  statistics, anti-diagonal alpha/beta sweeps, fused logits gradient).

Inputs are stacked log-mel frames ``[B, T, 240]`` (80 mels x 3, the MLPerf feature
front-end); labels are character ids ``0..vocab-2`` with ``blank = vocab - 1``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd import ops


@dataclass
class RNNTConfig:
    in_features: int = 240
    vocab: int = 29                 # 28 characters + blank
    enc_hidden: int = 1024
    enc_pre_layers: int = 2
    enc_post_layers: int = 3
    stack_time: int = 2
    pred_hidden: int = 320
    pred_layers: int = 2
    joint_hidden: int = 512
    dropout: float = 0.32

    @property
    def blank(self) -> int:
        return self.vocab - 1

    @classmethod
    def tiny(cls, **kw):
        base = dict(in_features=24, vocab=8, enc_hidden=32, enc_pre_layers=1, enc_post_layers=1, pred_hidden=24,
                    pred_layers=1, joint_hidden=32, dropout=0.0)
        base.update(kw)
        return cls(**base)


def run_lstm(m: nn.LSTM, x: torch.Tensor, hx=None):
    """Run ``m`` with fp32 math on the GPU when its parameters are bf16.

    MIOpen's fused RNN kernels support fp32 / fp16 but not bf16; a bf16 ``nn.LSTM`` falls back
    to PyTorch's per-time-step GEMM + cell kernels (measured on MI355X for the MLPerf encoder
    layer, 32 x 400 frames: 163 ms fwd+bwd in bf16 vs 40 ms through MIOpen in fp32).  The bf16
    weights are cast per call (a few MB, differentiable), the recurrence runs in MIOpen fp32,
    and the output returns in the model dtype."""
    if not (x.is_cuda and m.weight_ih_l0.dtype == torch.bfloat16):
        return m(x, hx)
    L = m.num_layers * (2 if m.bidirectional else 1)
    B = x.shape[0] if m.batch_first else x.shape[1]
    if hx is None:
        z = torch.zeros(L, B, m.hidden_size, device=x.device, dtype=torch.float32)
        hx = (z, z)
    else:
        hx = (hx[0].float(), hx[1].float())
    w = [p.float() for p in m._flat_weights]
    out, h, c = torch._VF.lstm(x.float(), hx, w, m.bias, m.num_layers, float(m.dropout), m.training,
                               m.bidirectional, m.batch_first)
    return out.to(x.dtype), (h, c)


class StackTime(nn.Module):
    """[B, T, C] -> [B, ceil(T/f), C*f] (frame stacking; lengths divided by f)."""

    def __init__(self, factor: int):
        super().__init__()
        self.f = factor

    def forward(self, x, lengths):
        B, T, C = x.shape
        pad = (-T) % self.f
        if pad:
            x = F.pad(x, (0, 0, 0, pad))
        return x.reshape(B, (T + pad) // self.f, C * self.f), (lengths + self.f - 1) // self.f


class RNNT(nn.Module):
    def __init__(self, cfg: RNNTConfig = None, device=None, dtype=torch.bfloat16):
        super().__init__()
        cfg = cfg or RNNTConfig()
        self.cfg = cfg
        kw = dict(device=device, dtype=dtype)
        h = cfg.enc_hidden
        self.pre_rnn = nn.LSTM(cfg.in_features, h, cfg.enc_pre_layers, batch_first=True, dropout=cfg.dropout
                               if cfg.enc_pre_layers > 1 else 0.0, **kw)
        self.stack = StackTime(cfg.stack_time)
        self.post_rnn = nn.LSTM(h * cfg.stack_time, h, cfg.enc_post_layers, batch_first=True,
                                dropout=cfg.dropout if cfg.enc_post_layers > 1 else 0.0, **kw)
        self.embed = nn.Embedding(cfg.vocab - 1, cfg.pred_hidden, **kw)      # blank is never an input
        self.pred_rnn = nn.LSTM(cfg.pred_hidden, cfg.pred_hidden, cfg.pred_layers, batch_first=True,
                                dropout=cfg.dropout if cfg.pred_layers > 1 else 0.0, **kw)
        self.enc_proj = nn.Linear(h, cfg.joint_hidden, **kw)
        self.pred_proj = nn.Linear(cfg.pred_hidden, cfg.joint_hidden, **kw)
        self.joint_out = nn.Linear(cfg.joint_hidden, cfg.vocab, **kw)
        self.dtype = dtype

    # ------------------------------------------------------------------ networks
    def encode(self, feats: torch.Tensor, lengths: torch.Tensor):
        x, _ = run_lstm(self.pre_rnn, feats.to(self.dtype))
        x, lengths = self.stack(x, lengths)
        x, _ = run_lstm(self.post_rnn, x)
        return x, lengths

    def predict(self, labels: torch.Tensor, state=None, prepend_sos: bool = True):
        """labels [B, U] -> prediction outputs [B, U+1, H] (the first step sees a zero SOS)."""
        e = self.embed(labels.clamp(min=0, max=self.cfg.vocab - 2))
        if prepend_sos:
            e = F.pad(e, (0, 0, 1, 0))
        g, state = run_lstm(self.pred_rnn, e, state)
        return g, state

    def joint(self, f: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
        """f [B, T, H_enc], g [B, U+1, H_pred] -> logits [B, T, U+1, V]."""
        h = F.relu(self.enc_proj(f).unsqueeze(2) + self.pred_proj(g).unsqueeze(1))
        if self.training and self.cfg.dropout:
            h = F.dropout(h, self.cfg.dropout)
        return self.joint_out(h)

    def forward(self, feats, feat_lengths, labels, label_lengths):
        """Training: mean transducer loss over the batch."""
        f, f_len = self.encode(feats, feat_lengths)
        g, _ = self.predict(labels)
        logits = self.joint(f, g)
        return ops.rnnt_loss(logits, labels, f_len, label_lengths, blank=self.cfg.blank)

    # ------------------------------------------------------------------ decoding
    @torch.no_grad()
    def greedy_decode(self, feats, feat_lengths, max_symbols_per_step: int = 30) -> List[List[int]]:
        """Batched greedy search: every utterance advances one encoder frame per outer step
        and emits up to ``max_symbols_per_step`` labels at that frame.  Emissions are
        recorded on the device (one [B, T * max_symbols] buffer); the only host round trip
        per symbol step is the "anyone still emitting?" test."""
        f, f_len = self.encode(feats, feat_lengths)
        B, T, _ = f.shape
        fp = self.enc_proj(f)
        blank = self.cfg.blank
        dev = f.device
        cap = T * max_symbols_per_step
        out = torch.full((B, cap), -1, dtype=torch.long, device=dev)
        count = torch.zeros(B, dtype=torch.long, device=dev)
        rows = torch.arange(B, device=dev)
        g, state = run_lstm(self.pred_rnn, torch.zeros(B, 1, self.cfg.pred_hidden, device=dev, dtype=self.dtype))
        gp = self.pred_proj(g[:, 0])
        f_len = f_len.to(dev)
        for t in range(T):
            active = t < f_len
            for _ in range(max_symbols_per_step):
                k = self.joint_out(F.relu(fp[:, t] + gp)).float().argmax(-1)
                emit = active & (k != blank)
                if not bool(emit.any()):
                    break
                out[rows, count.clamp(max=cap - 1)] = torch.where(emit, k, out[rows, count.clamp(max=cap - 1)])
                count += emit.long()
                g_new, st_new = run_lstm(self.pred_rnn, self.embed(k.clamp(max=self.cfg.vocab - 2)).unsqueeze(1),
                                         state)
                m = emit.view(1, B, 1).to(st_new[0].dtype)
                state = tuple(s_new * m + s_old * (1 - m) for s_new, s_old in zip(st_new, state))
                gp = torch.where(emit[:, None], self.pred_proj(g_new[:, 0]), gp)
        out, count = out.cpu(), count.cpu()
        return [out[b, :int(count[b])].tolist() for b in range(B)]


def rnnt_mlperf(device=None, dtype=torch.bfloat16) -> RNNT:
    return RNNT(RNNTConfig(), device=device, dtype=dtype)


def synthetic_speech_batch(B: int, T: int = 400, U: int = 60, cfg: RNNTConfig = None, device=None,
                           generator: torch.Generator = None):
    cfg = cfg or RNNTConfig()
    g = generator or torch.Generator().manual_seed(0)
    feats = torch.randn(B, T, cfg.in_features, generator=g)
    feat_len = torch.randint(T * 3 // 4, T + 1, (B,), generator=g)
    feat_len[0] = T
    lab_len = torch.randint(max(1, U // 2), U + 1, (B,), generator=g)
    lab_len[0] = U
    labels = torch.randint(0, cfg.vocab - 1, (B, U), generator=g)
    if device is not None:
        feats, labels = feats.to(device), labels.to(device)
    return feats, feat_len, labels, lab_len
