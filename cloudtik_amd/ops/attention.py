"""Fused attention front-end (HIP MFMA kernels in csrc/attention.hip).

Two entry points:

* :func:`attention_packed` -- BERT/GPT path: takes the packed QKV projection output
  ``[B, S, 3*H*64]`` (no permute/contiguous copies: the kernel reads Q, K, V through
  strides), returns ``[B, S, H*64]`` ready for the output projection, and its backward
  writes dQ, dK, dV into ONE packed ``[B, S, 3*H*64]`` gradient so the QKV projection's
  backward is a single GEMM.
* :func:`attention` -- generic ``[B, H, S, D]`` tensors (torch SDPA layout).

``key_bias`` is an additive fp32 ``[B, Sk]`` per-key bias (HF BERT: ``(1 - mask) * -10000``).
"""
from __future__ import annotations

import math

import torch

from . import reference as ref


def _ops():
    from cloudtik_amd import ops
    return ops


class _AttnPackedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, H, key_bias, scale, p, seed, offset, causal):
        B, S, W = qkv.shape
        D = W // (3 * H)
        v5 = qkv.view(B, S, 3, H, D)
        q, k, v = v5[:, :, 0], v5[:, :, 1], v5[:, :, 2]
        o = torch.empty(B, S, H, D, dtype=qkv.dtype, device=qkv.device)
        lse = _ops().require_native().attn_fwd(q, k, v, o, key_bias, scale, p, seed, offset, causal)
        ctx.save_for_backward(qkv, o, lse, key_bias if key_bias is not None else torch.empty(0))
        ctx.cfg = (H, scale, p, seed, offset, causal, key_bias is not None)
        return o.view(B, S, H * D)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, kb = ctx.saved_tensors
        H, scale, p, seed, offset, causal, has_kb = ctx.cfg
        B, S, W = qkv.shape
        D = W // (3 * H)
        v5 = qkv.view(B, S, 3, H, D)
        dqkv = torch.empty_like(qkv)
        d5 = dqkv.view(B, S, 3, H, D)
        do4 = do.contiguous().view(B, S, H, D)
        _ops().require_native().attn_bwd(v5[:, :, 0], v5[:, :, 1], v5[:, :, 2], o, do4,
                                         d5[:, :, 0], d5[:, :, 1], d5[:, :, 2],
                                         kb if has_kb else None, lse, scale, p, seed, offset, causal)
        return dqkv, None, None, None, None, None, None, None


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, key_bias, scale, p, seed, offset, causal):
        # q, k, v: [B, S, H, D] views
        B, Sq, H, D = q.shape
        o = torch.empty(B, Sq, H, D, dtype=q.dtype, device=q.device)
        lse = _ops().require_native().attn_fwd(q, k, v, o, key_bias, scale, p, seed, offset, causal)
        ctx.save_for_backward(q, k, v, o, lse, key_bias if key_bias is not None else torch.empty(0))
        ctx.cfg = (scale, p, seed, offset, causal, key_bias is not None)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kb = ctx.saved_tensors
        scale, p, seed, offset, causal, has_kb = ctx.cfg
        dq = torch.empty(q.shape, dtype=q.dtype, device=q.device)
        dk = torch.empty(k.shape, dtype=k.dtype, device=k.device)
        dv = torch.empty(v.shape, dtype=v.dtype, device=v.device)
        _ops().require_native().attn_bwd(q, k, v, o, do.contiguous(), dq, dk, dv,
                                         kb if has_kb else None, lse, scale, p, seed, offset, causal)
        return dq, dk, dv, None, None, None, None, None, None


def _native_ok(t, D):
    return t.is_cuda and t.dtype == torch.bfloat16 and D == 64


def attention_packed(qkv, num_heads, key_bias=None, p=0.0, training=True, scale=None,
                     causal=False):
    """qkv: [B, S, 3*H*D] -> [B, S, H*D]."""
    B, S, W = qkv.shape
    D = W // (3 * num_heads)
    scale = float(scale if scale is not None else 1.0 / math.sqrt(D))
    p = float(p) if training else 0.0
    ops = _ops()
    seed, offset = ops._rng.next(B * num_heads * S * S) if p > 0 else (0, 0)
    if key_bias is not None:
        key_bias = key_bias.float().contiguous()
    if ops._use_native(qkv) and _native_ok(qkv, D) and (p == 0 or S % 2 == 0):
        return _AttnPackedFn.apply(qkv.contiguous(), num_heads, key_bias, scale, p, seed, offset, bool(causal))
    v5 = qkv.view(B, S, 3, num_heads, D).permute(2, 0, 3, 1, 4)
    o = ref.attention(v5[0], v5[1], v5[2], key_bias, p, seed, offset, scale, causal)
    return o.permute(0, 2, 1, 3).reshape(B, S, num_heads * D)


def attention(q, k, v, key_bias=None, p=0.0, scale=None, causal=False):
    """q, k, v: [B, H, S, D] -> [B, H, Sq, D]."""
    B, H, Sq, D = q.shape
    Sk = k.shape[2]
    scale = float(scale if scale is not None else 1.0 / math.sqrt(D))
    ops = _ops()
    seed, offset = ops._rng.next(B * H * Sq * Sk) if p > 0 else (0, 0)
    if key_bias is not None:
        key_bias = key_bias.float().contiguous()
    if ops._use_native(q) and _native_ok(q, D) and (p == 0 or Sk % 2 == 0):
        o = _AttnFn.apply(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), key_bias, scale,
                          float(p), seed, offset, bool(causal))
        return o.transpose(1, 2)
    return ref.attention(q, k, v, key_bias, p, seed, offset, scale, causal)


def attention_relbias(q, k, v, rel_bias, rel_base: int, key_bias=None, scale: float = 1.0, causal: bool = False):
    """Inference attention with a relative-position bias (T5): q/k/v ``[B, S, H, D]``,
    ``rel_bias [H, L]`` adds ``rel_bias[h, k - q + rel_base]`` to every score (natural-log
    units), ``key_bias [B, Sk]`` masks keys.  HIP MFMA kernel on the GPU (bf16, D = 64);
    fp32 PyTorch reference elsewhere.  Forward only."""
    B, Sq, H, D = q.shape
    Sk = k.shape[1]
    if (q.is_cuda and q.dtype == torch.bfloat16 and D == 64 and rel_bias.shape[1] <= 4096
            and _ops().native_available()):
        o = torch.empty_like(q)
        kb = key_bias.float().contiguous() if key_bias is not None else None
        _ops().require_native().attn_fwd_relbias(q, k, v, o, kb, rel_bias.float().contiguous(), int(rel_base),
                                                 float(scale), bool(causal))
        return o
    idx = (torch.arange(Sk, device=q.device)[None, :] - torch.arange(Sq, device=q.device)[:, None] + rel_base)
    bias = rel_bias.float()[:, idx.clamp(0, rel_bias.shape[1] - 1)][None]            # [1, H, Sq, Sk]
    if key_bias is not None:
        bias = bias + key_bias.float()[:, None, None, :]
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale + bias
    if causal:
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), v.float()).to(q.dtype)
