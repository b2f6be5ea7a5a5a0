"""Plain-PyTorch reference implementations of every cloudtik_amd HIP op.

Used (a) as the CPU execution path and (b) as the fp32 oracle in the GPU numerics
tests.  The dropout masks are bit-identical to the kernels': both evaluate the same
counter-based hash stream (``common.h: dropout_bits8``), so a CPU run and a GPU run of the
same model with the same seed drop the same elements.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

M32 = np.uint64(0xFFFFFFFF)
ACT_NONE, ACT_GELU, ACT_RELU = 0, 1, 2


def _mix32(x):
    """common.h mix32 on uint64 arrays holding uint32 values."""
    x = x ^ (x >> np.uint64(16))
    x = (x * np.uint64(0x7FEB352D)) & M32
    x = x ^ (x >> np.uint64(15))
    x = (x * np.uint64(0x846CA68B)) & M32
    return x ^ (x >> np.uint64(16))


def _dropout_key(seed: int, offset: int) -> int:
    def m(x):
        return int(_mix32(np.array([x & 0xFFFFFFFF], dtype=np.uint64))[0])
    k = m(((offset >> 32) + 0x632BE5AB) & 0xFFFFFFFF)
    k = m(k ^ (offset & 0xFFFFFFFF))
    k = m(k ^ ((seed >> 32) & 0xFFFFFFFF))
    return m(k ^ (seed & 0xFFFFFFFF))


def dropout_threshold(p: float) -> int:
    t = float(p) * 4294967296.0
    return 0xFFFFFFFF if t >= 4294967295.0 else int(t)


def dropout_keep_mask(n: int, p: float, seed: int, offset: int) -> torch.Tensor:
    """Boolean keep-mask of ``n`` elements (n % 8 == 0), identical to the HIP kernels
    (common.h dropout_bits8: one 16-bit uniform per element from a hash of the pair counter)."""
    assert n % 8 == 0
    seed &= 0xFFFFFFFFFFFFFFFF
    offset &= 0xFFFFFFFFFFFFFFFF
    v = np.arange(n // 8, dtype=np.uint64)
    key = np.uint64(_dropout_key(seed, offset)) ^ _mix32((v >> np.uint64(30)) & M32)
    t16 = np.uint64(dropout_threshold(p) >> 16)
    out = np.empty((n // 8, 8), dtype=bool)
    for j in range(4):
        ctr = ((v << np.uint64(2)) | np.uint64(j)) & M32
        r = _mix32(((((ctr + key) & M32) * np.uint64(0x9E3779B1)) & M32) ^ key)
        out[:, 2 * j] = (r & np.uint64(0xFFFF)) >= t16
        out[:, 2 * j + 1] = (r >> np.uint64(16)) >= t16
    return torch.from_numpy(out.reshape(-1))


def dropout(x: torch.Tensor, p: float, seed: int, offset: int) -> torch.Tensor:
    if p <= 0.0:
        return x
    keep = dropout_keep_mask(x.numel(), p, seed, offset).to(x.device).view_as(x)
    return torch.where(keep, x * (1.0 / (1.0 - p)), torch.zeros_like(x))


def _round(x: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    return x.to(like.dtype).to(torch.float32) if like.dtype != torch.float32 else x


def layer_norm(x, gamma, beta=None, eps=1e-12, bias=None, residual=None, p=0.0, seed=0,
               offset=0, rms=False):
    """y = LN(residual + dropout(x + bias)); returns (y, s) with s the LN input."""
    xf = x.float()
    if bias is not None:
        xf = xf + bias.float()
    if p > 0.0:
        xf = dropout(xf, p, seed, offset)
    if residual is not None:
        xf = xf + residual.float()
    s = _round(xf, x)
    if rms:
        var = (s * s).mean(-1, keepdim=True)
        y = s * torch.rsqrt(var + eps) * gamma.float()
    else:
        mean = s.mean(-1, keepdim=True)
        var = ((s - mean) ** 2).mean(-1, keepdim=True)
        y = (s - mean) * torch.rsqrt(var + eps) * gamma.float()
        if beta is not None:
            y = y + beta.float()
    return y.to(x.dtype), s.to(x.dtype)


def bias_act(z, bias=None, act=ACT_GELU):
    t = z.float()
    if bias is not None:
        t = t + bias.float()
    if act == ACT_GELU:
        t = F.gelu(t)
    elif act == ACT_RELU:
        t = F.relu(t)
    return t.to(z.dtype)


def embedding3(ids, tt, W, P=None, T=None):
    out = W.float()[ids]
    if P is not None:
        out = out + P.float()[: ids.shape[1]].unsqueeze(0)
    if T is not None:
        out = out + T.float()[tt if tt is not None else torch.zeros_like(ids)]
    return out.to(W.dtype)


def cross_entropy(logits, labels, V=None, ignore_index=-100, label_smoothing=0.0):
    """Mean CE over valid rows of logits[:, :V] (fp32 math)."""
    V = V or logits.shape[-1]
    return F.cross_entropy(logits[:, :V].float(), labels, ignore_index=ignore_index,
                           label_smoothing=label_smoothing)


def _hash_u32(x):
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x = x ^ (x >> 16)
    return x


def attn_dropout_keep(B, H, Sq, Sk, p, seed, offset):
    """Keep mask [B, H, Sq, Sk] identical to the attention kernels' hash-based stream."""
    idx = np.arange(B * H * Sq * Sk, dtype=np.uint64).reshape(B, H, Sq, Sk)
    pair = idx >> np.uint64(1)
    half = (idx & np.uint64(1)).astype(np.uint64)
    s_lo = np.uint64(seed & 0xFFFFFFFF)
    s_hi = np.uint64((seed >> 32) & 0xFFFFFFFF)
    off = np.uint64(offset & 0xFFFFFFFF)
    base = _hash_u32((s_lo ^ (s_hi * np.uint64(0x85EBCA6B) & M32) ^ (off * np.uint64(0xC2B2AE35) & M32)) & M32)
    r = _hash_u32(((pair & M32) ^ base) & M32)
    r16 = (r >> (half * np.uint64(16))) & np.uint64(0xFFFF)
    thr = np.uint64(min(65535, int(round(p * 65536.0))))
    return torch.from_numpy(r16 >= thr)


def attention(q, k, v, key_bias=None, p=0.0, seed=0, offset=0, scale=None, causal=False):
    """q,k,v: [B, H, S, D]; key_bias: additive [B, Sk] (fp32). Returns [B, H, Sq, D]."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if key_bias is not None:
        s = s + key_bias.float()[:, None, None, :]
    if causal:
        Sq, Sk = s.shape[-2:]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).triu(1)
        s = s.masked_fill(m, float("-inf"))
    pr = torch.softmax(s, -1)
    if p > 0.0:
        keep = attn_dropout_keep(*s.shape, p, seed, offset).to(s.device)
        pr = torch.where(keep, pr / (1.0 - p), torch.zeros_like(pr))
    return torch.matmul(pr, v.float()).to(q.dtype)
