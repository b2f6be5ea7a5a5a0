"""Rotary position embedding with the HIP kernel (csrc/rope.hip).

``apply_rotary(q, k, cos, sin, positions=None, neox=True)`` rotates q ([B, S, H, D] or
[T, H, D], bf16) and optionally k in place-free fashion (returns new tensors) with autograd.
``rotary_cache(max_pos, D, base)`` builds the fp32 cos/sin tables [P, D/2].
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def rotary_cache(max_positions: int, head_dim: int, base: float = 10000.0, device=None,
                 scaling: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(max_positions, dtype=torch.float64) / scaling
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def rope_reference(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, positions: Optional[torch.Tensor] = None,
                   neox: bool = True, inverse: bool = False) -> torch.Tensor:
    """fp32 reference on [T, H, D] (positions [T] or implicit 0..T-1 per sequence of length P)."""
    T, H, D = x.shape
    pos = positions if positions is not None else torch.arange(T, device=x.device)
    c = cos[pos].float()[:, None, :]
    s = sin[pos].float()[:, None, :]
    if inverse:
        s = -s
    xf = x.float()
    if neox:
        x1, x2 = xf[..., :D // 2], xf[..., D // 2:]
        return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
    x1, x2 = xf[..., 0::2], xf[..., 1::2]
    out = torch.empty_like(xf)
    out[..., 0::2] = x1 * c - x2 * s
    out[..., 1::2] = x2 * c + x1 * s
    return out


def _as_thd(x: torch.Tensor):
    if x.dim() == 4:            # [B, S, H, D]
        B, S, H, D = x.shape
        return x.reshape(B * S, H, D), S
    return x, x.shape[0]


def _native():
    from cloudtik_amd import ops
    return ops.require_native()


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, cos, sin, positions, neox):
        q3, S = _as_thd(q)
        qo = q3.contiguous().clone()
        ko = None
        if k is not None:
            k3, _ = _as_thd(k)
            ko = k3.contiguous().clone()
        _native().rope(qo, ko, cos, sin, positions, S, neox, False)
        ctx.save_for_backward(cos, sin, positions if positions is not None else torch.empty(0))
        ctx.has_pos = positions is not None
        ctx.neox, ctx.S = neox, S
        ctx.qshape, ctx.kshape = q.shape, (k.shape if k is not None else None)
        return qo.view(q.shape), (ko.view(k.shape) if ko is not None else None)

    @staticmethod
    def backward(ctx, dq, dk):
        cos, sin, pos = ctx.saved_tensors
        pos = pos if ctx.has_pos else None
        dq3 = dq.reshape(-1, ctx.qshape[-2], ctx.qshape[-1]).contiguous().clone()
        dk3 = None
        if ctx.kshape is not None:
            if dk is None:
                dk = torch.zeros(ctx.kshape, dtype=dq.dtype, device=dq.device)
            dk3 = dk.reshape(-1, ctx.kshape[-2], ctx.kshape[-1]).contiguous().clone()
        _native().rope(dq3, dk3, cos, sin, pos, ctx.S, ctx.neox, True)
        return (dq3.view(ctx.qshape), dk3.view(ctx.kshape) if dk3 is not None else None, None, None, None, None)


def apply_rotary(q: torch.Tensor, k: Optional[torch.Tensor], cos: torch.Tensor, sin: torch.Tensor,
                 positions: Optional[torch.Tensor] = None, neox: bool = True):
    """Rotate q (and k) by their positions.  q/k: [B, S, H, D] or [T, H, D] bf16."""
    from cloudtik_amd import ops
    if q.is_cuda and q.dtype == torch.bfloat16 and ops._use_native(q):
        if positions is not None:
            positions = positions.reshape(-1).contiguous()
        return _RopeFn.apply(q, k, cos, sin, positions, neox)
    q3, S = _as_thd(q)
    pos = positions.reshape(-1) if positions is not None else torch.arange(q3.shape[0], device=q.device) % S
    qo = rope_reference(q3, cos, sin, pos, neox).to(q.dtype).view(q.shape)
    ko = None
    if k is not None:
        k3, _ = _as_thd(k)
        ko = rope_reference(k3, cos, sin, pos, neox).to(k.dtype).view(k.shape)
    return qo, ko
