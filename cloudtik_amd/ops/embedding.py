"""DLRM sparse ops: multi-table EmbeddingBag and the dot-product interaction, with autograd
(HIP kernels in csrc/embedding.hip; torch references for CPU).

Reference: DLRM dlrm_s_pytorch.py:267-269 (one nn.EmbeddingBag per table, sum pooling),
:407-418 (interact_features), IPEX SplitSGD / fused embedding update.

``EmbeddingBagCollection`` keeps all tables in one fp32 [sum(V_t), E] parameter.  Its
backward either returns a dense gradient (regular optimizers) or, when ``sparse_lr`` is set,
applies ``w[row] -= lr * grad`` to the touched rows inside the backward kernel and reports
no gradient -- the DLRM-style sparse update that never materialises a dense 10^7 x E
gradient.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F


def _native():
    from cloudtik_amd import ops
    return ops.require_native()


def _use_native(*ts) -> bool:
    from cloudtik_amd import ops
    return ops._use_native(*ts)


def pack_bags(indices: Sequence[torch.Tensor], offsets: Sequence[torch.Tensor], batch: int):
    """Per-table (indices [n_t], offsets [B] start positions) -> one CSR over T*B bags."""
    idx = torch.cat([i.reshape(-1) for i in indices])
    parts, base = [], 0
    for i, o in zip(indices, offsets):
        parts.append(o.reshape(-1).to(torch.int64) + base)
        base += i.numel()
    offs = torch.cat(parts + [torch.tensor([base], dtype=torch.int64, device=idx.device)])
    assert offs.numel() == len(indices) * batch + 1
    return idx, offs


def embedding_bag_reference(W, row_base, idx, offs, B, psw=None, mean=False):
    T = row_base.numel()
    E = W.shape[1]
    bag_of = torch.repeat_interleave(torch.arange(T * B, device=W.device), offs[1:] - offs[:-1])
    t_of = bag_of // B
    rows = W[row_base[t_of] + idx].float()
    if psw is not None:
        rows = rows * psw[:, None]
    flat = torch.zeros(T * B, E, dtype=torch.float32, device=W.device)   # bags are table-major
    flat.index_add_(0, bag_of, rows)
    if mean:
        cnt = (offs[1:] - offs[:-1]).clamp(min=1).float()
        flat = flat / cnt[:, None]
    return flat.view(T, B, E).transpose(0, 1).contiguous()


class _EmbBagFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, W, row_base, idx, offs, psw, B, mean, bf16_out, sparse_lr):
        out = _native().embbag_fwd(W, row_base, idx, offs, psw, B, mean, bf16_out)
        ctx.save_for_backward(W, row_base, idx, offs, psw if psw is not None else torch.empty(0))
        ctx.B, ctx.mean, ctx.sparse_lr, ctx.has_psw = B, mean, sparse_lr, psw is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        W, row_base, idx, offs, psw = ctx.saved_tensors
        psw = psw if ctx.has_psw else None
        gout = gout.contiguous()
        dpsw = torch.empty_like(psw) if (psw is not None and ctx.needs_input_grad[4]) else None
        if ctx.sparse_lr:
            _native().embbag_bwd(gout, W, None, row_base, idx, offs, psw, dpsw, ctx.mean, float(ctx.sparse_lr))
            dW = None
        else:
            dW = torch.zeros_like(W)
            _native().embbag_bwd(gout, W, dW, row_base, idx, offs, psw, dpsw, ctx.mean, 0.0)
        return dW, None, None, None, dpsw, None, None, None, None


def embedding_bag(W, row_base, idx, offs, batch: int, per_sample_weights=None, mean: bool = False,
                  bf16_out: bool = False, sparse_lr: float = 0.0):
    if W.is_cuda and _use_native(W):
        return _EmbBagFn.apply(W, row_base, idx, offs, per_sample_weights, batch, mean, bf16_out, sparse_lr)
    out = embedding_bag_reference(W, row_base, idx, offs, batch, per_sample_weights, mean)
    return out.to(torch.bfloat16) if bf16_out else out


class EmbeddingBagCollection(nn.Module):
    """All sparse feature tables of a DLRM in one parameter; forward -> [B, T, E]."""

    def __init__(self, num_embeddings: List[int], dim: int, mode: str = "sum", device=None,
                 bf16_out: bool = False, sparse_lr: float = 0.0):
        super().__init__()
        if mode not in ("sum", "mean"):
            raise ValueError("mode must be sum or mean")
        self.num_embeddings = list(num_embeddings)
        self.dim = dim
        self.mean = mode == "mean"
        self.bf16_out = bf16_out
        self.sparse_lr = sparse_lr
        total = sum(num_embeddings)
        w = torch.empty(total, dim, dtype=torch.float32, device=device)
        base = 0
        with torch.no_grad():
            for n in num_embeddings:       # DLRM init: U(-sqrt(1/n), sqrt(1/n)) per table
                b = math.sqrt(1.0 / n)
                w[base:base + n].uniform_(-b, b)
                base += n
        self.weight = nn.Parameter(w)
        rb = torch.tensor([0] + list(torch.tensor(num_embeddings).cumsum(0)[:-1].tolist()), dtype=torch.int64)
        self.register_buffer("row_base", rb.to(device), persistent=False)

    def forward(self, indices: torch.Tensor, offsets: torch.Tensor, batch: int, per_sample_weights=None):
        return embedding_bag(self.weight, self.row_base, indices, offsets, batch, per_sample_weights,
                             self.mean, self.bf16_out, self.sparse_lr if self.training else 0.0)


# ---------------------------------------------------------------------- interaction
def interaction_reference(x: torch.Tensor, emb: torch.Tensor) -> torch.Tensor:
    B, E = x.shape
    V = torch.cat([x[:, None, :], emb], dim=1).float()
    Z = torch.bmm(V, V.transpose(1, 2))
    Fn = V.shape[1]
    li, lj = torch.tril_indices(Fn, Fn, offset=-1, device=x.device)
    return torch.cat([x.float(), Z[:, li, lj]], dim=1)


class _InteractFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, emb):
        x, emb = x.contiguous(), emb.contiguous()
        ctx.save_for_backward(x, emb)
        return _native().interact_fwd(x, emb)

    @staticmethod
    def backward(ctx, g):
        x, emb = ctx.saved_tensors
        dx, demb = _native().interact_bwd(g.contiguous(), x, emb)
        return dx, demb


def dot_interaction(x: torch.Tensor, emb: torch.Tensor) -> torch.Tensor:
    """[x, strictly-lower-triangle of [x;emb][x;emb]^T]  ->  [B, E + F(F-1)/2]."""
    if x.is_cuda and _use_native(x) and x.dtype == emb.dtype:
        return _InteractFn.apply(x, emb)
    return interaction_reference(x, emb).to(x.dtype)
