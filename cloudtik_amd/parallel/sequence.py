"""Sequence (context) parallelism for long sequences (ring attention and
Ulysses, both reusing the attention kernel with an LSE merge).

The sequence dimension is sharded over the ranks of ``group``: rank r holds tokens
[r*S/P, (r+1)*S/P) of q, k and v (layout [B, S/P, H, D]).

* ``ulysses_attention``: all-to-all re-shards sequence <-> heads (every rank gets the whole
  sequence for H/P heads), runs ordinary attention locally, and all-to-alls back.  Two
  all-to-alls of the activations per direction; needs H divisible by P.
* ``ring_attention``: K/V blocks travel around the ring (send to r+1, receive from r-1 with
  one batched P2P per step, issued BEFORE the block's compute so the transfer overlaps it);
  each rank merges the partial block outputs with their log-sum-exp.  The backward pass
  sends the K/V blocks around again together with their dK/dV accumulators, and recomputes
  each block's probabilities from the GLOBAL log-sum-exp -- exactly what the HIP backward
  kernel does given the final O and LSE -- so memory stays O(S/P) per rank.  With
  ``causal=True`` blocks above the diagonal are skipped and the diagonal block is causal.

On MI355X (bf16, head dim 64) the per-block work is the MFMA attention kernel pair
(``attn_fwd`` returns the log2-domain LSE the merge needs); elsewhere a fp32 PyTorch
block implementation with identical semantics is used (this is what the gloo tests run).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.distributed as dist

LN2 = math.log(2.0)


# --------------------------------------------------------------------------- blocks
def _native_ok(q: torch.Tensor) -> bool:
    if not (q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] == 64):
        return False
    from cloudtik_amd import ops
    return ops.native_available()


def block_forward(q, k, v, scale: float, causal: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """q [B, Sq, H, D], k/v [B, Sk, H, D] -> (o [B, Sq, H, D] fp32, lse [B, H, Sq] natural log)."""
    B, Sq, H, D = q.shape
    if _native_ok(q):
        from cloudtik_amd import ops
        o = torch.empty_like(q)
        lse2 = ops.require_native().attn_fwd(q, k, v, o, None, scale, 0.0, 0, 0, causal)
        return o.float(), lse2.view(B, H, Sq) * LN2
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale
    if causal:
        s = s.masked_fill(torch.ones(Sq, k.shape[1], dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    p = torch.exp(s - lse[..., None])
    return torch.einsum("bhqk,bkhd->bqhd", p, v.float()), lse


def block_backward(q, k, v, o, do, lse, scale: float, causal: bool):
    """Gradients of one (q-block, kv-block) pair given the GLOBAL output ``o`` and ``lse``."""
    B, Sq, H, D = q.shape
    if _native_ok(q):
        from cloudtik_amd import ops
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        lse2 = (lse / LN2).reshape(B * H, Sq).contiguous()
        ops.require_native().attn_bwd(q, k, v, o.to(q.dtype).contiguous(), do.to(q.dtype).contiguous(), dq, dk, dv,
                                      None, lse2, scale, 0.0, 0, 0, causal)
        return dq.float(), dk.float(), dv.float()
    qf, kf, vf, of, dof = q.float(), k.float(), v.float(), o.float(), do.float()
    s = torch.einsum("bqhd,bkhd->bhqk", qf, kf) * scale
    if causal:
        s = s.masked_fill(torch.ones(Sq, k.shape[1], dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    p = torch.exp(s - lse[..., None])
    dv = torch.einsum("bhqk,bqhd->bkhd", p, dof)
    dp = torch.einsum("bqhd,bkhd->bhqk", dof, vf)
    delta = (dof * of).sum(-1).permute(0, 2, 1)                       # [B, H, Sq]
    ds = p * (dp - delta[..., None]) * scale
    return torch.einsum("bhqk,bkhd->bqhd", ds, kf), torch.einsum("bhqk,bqhd->bkhd", ds, qf), dv


# --------------------------------------------------------------------------- ring
def _ring_exchange(tensors, group, rank, world):
    """Send ``tensors`` to rank+1, receive the same shapes from rank-1 (one batched P2P)."""
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    g_nxt = dist.get_global_rank(group, nxt) if group is not None else nxt
    g_prv = dist.get_global_rank(group, prv) if group is not None else prv
    recv = [torch.empty_like(t) for t in tensors]
    ops_ = [dist.P2POp(dist.isend, t.contiguous(), g_nxt, group) for t in tensors] + \
           [dist.P2POp(dist.irecv, r, g_prv, group) for r in recv]
    return recv, dist.batch_isend_irecv(ops_)


def _wait(reqs):
    for r in reqs:
        r.wait()


class _RingAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal, group):
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        B, S, H, D = q.shape
        o = torch.zeros(B, S, H, D, dtype=torch.float32, device=q.device)
        lse = torch.full((B, H, S), float("-inf"), dtype=torch.float32, device=q.device)
        kv = (k.contiguous(), v.contiguous())
        for step in range(world):
            src = (rank - step) % world                       # owner of the kv block held now
            reqs = None
            if step + 1 < world:
                nxt_kv, reqs = _ring_exchange(kv, group, rank, world)
            if not (causal and src > rank):
                ob, lb = block_forward(q, kv[0], kv[1], scale, causal and src == rank)
                new = torch.logaddexp(lse, lb)
                w_old = torch.exp(lse - new).nan_to_num(0.0).permute(0, 2, 1)[..., None]
                w_new = torch.exp(lb - new).nan_to_num(0.0).permute(0, 2, 1)[..., None]
                o = o * w_old + ob * w_new
                lse = new
            if reqs is not None:
                _wait(reqs)
                kv = nxt_kv
        out = o.to(q.dtype)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.scale, ctx.causal, ctx.group = scale, causal, group
        return out

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        group = ctx.group
        world = dist.get_world_size(group)
        rank = dist.get_rank(group)
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        # the kv block and its gradient accumulators travel together
        kv = [k.contiguous(), v.contiguous(), torch.zeros(k.shape, dtype=torch.float32, device=k.device),
              torch.zeros(v.shape, dtype=torch.float32, device=v.device)]
        for step in range(world):
            src = (rank - step) % world
            if not (ctx.causal and src > rank):
                dqb, dkb, dvb = block_backward(q, kv[0], kv[1], o, do, lse, ctx.scale, ctx.causal and src == rank)
                dq += dqb
                kv[2] = kv[2] + dkb
                kv[3] = kv[3] + dvb
            # P sends in total: after the last one every block (with its finished dK/dV)
            # is back on its owner
            kv, reqs = _ring_exchange(kv, group, rank, world)
            _wait(reqs)
        return dq.to(q.dtype), kv[2].to(k.dtype), kv[3].to(v.dtype), None, None, None


def ring_attention(q, k, v, group=None, scale: Optional[float] = None, causal: bool = False):
    """Context-parallel attention over sequence shards [B, S/P, H, D] (returns the local
    shard of the output)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return _single(q, k, v, scale, causal)
    return _RingAttention.apply(q, k, v, float(scale), bool(causal), group)


# --------------------------------------------------------------------------- Ulysses
class _AllToAll(torch.autograd.Function):
    """[B, S/P, H, D] -> [B, S, H/P, D] (``to_heads``) or the inverse; autograd = inverse."""

    @staticmethod
    def forward(ctx, x, group, to_heads):
        ctx.group, ctx.to_heads = group, to_heads
        return _a2a(x, group, to_heads)

    @staticmethod
    def backward(ctx, g):
        return _a2a(g.contiguous(), ctx.group, not ctx.to_heads), None, None


def _a2a(x, group, to_heads):
    P = dist.get_world_size(group)
    if to_heads:
        B, s, H, D = x.shape
        # split heads into P groups: send head-group j to rank j
        send = x.reshape(B, s, P, H // P, D).permute(2, 0, 1, 3, 4).contiguous()      # [P, B, s, H/P, D]
        recv = torch.empty_like(send)
        dist.all_to_all_single(recv, send, group=group)
        # recv[j] = rank j's sequence shard of my head group
        return recv.permute(1, 0, 2, 3, 4).reshape(B, P * s, H // P, D)
    B, S, h, D = x.shape
    s = S // P
    send = x.reshape(B, P, s, h, D).permute(1, 0, 2, 3, 4).contiguous()              # [P, B, s, h, D]
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    # recv[j] = my sequence shard of head group j
    return recv.permute(1, 2, 0, 3, 4).reshape(B, s, P * h, D)


def _single(q, k, v, scale, causal):
    if _native_ok(q):
        from cloudtik_amd import ops
        return ops.attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=scale,
                             causal=causal).transpose(1, 2)
    from cloudtik_amd.ops import reference as ref
    o = ref.attention(q.transpose(1, 2).float(), k.transpose(1, 2).float(), v.transpose(1, 2).float(),
                      scale=scale, causal=causal)
    return o.transpose(1, 2).to(q.dtype)


def ulysses_attention(q, k, v, group=None, scale: Optional[float] = None, causal: bool = False):
    """DeepSpeed-Ulysses-style attention over sequence shards [B, S/P, H, D]."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return _single(q, k, v, scale, causal)
    P = dist.get_world_size(group)
    if q.shape[2] % P:
        raise ValueError(f"Ulysses needs heads ({q.shape[2]}) divisible by the group size ({P})")
    qh, kh, vh = (_AllToAll.apply(t, group, True) for t in (q, k, v))
    oh = _single(qh, kh, vh, scale, causal)
    return _AllToAll.apply(oh.contiguous(), group, False)
