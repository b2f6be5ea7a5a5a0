"""T5 encoder-decoder (t5-small / base / large topologies).

Reference workload: the quickstart T5 inference (applications/ai/quickstart, HF
``T5ForConditionalGeneration``).  Random-init weights, same architecture:
pre-norm blocks with RMS LayerNorm (no mean, no bias), un-scaled attention with a learned
bucketed relative-position bias shared by all layers of a stack, ReLU (v1.0) or gated-GELU
(v1.1) feed-forward, tied input/output embeddings scaled by d_model^-0.5.

MI355X mapping: RMS norms run in the HIP LayerNorm kernel (``rms=True``); the relative
position bias is carried as one [H, Sq + Sk - 1] vector per stack (bias depends only on
key - query) and added inside the MFMA flash-attention kernel (``ops.attention_relbias``),
so inference never materialises an [H, Sq, Sk] bias; cross-attention uses the MFMA kernel
with the per-key padding mask; training self-attention (which needs the bias gradient) uses
SDPA with the gathered bias; the training loss is the fused linear + cross-entropy HIP
kernel over the 32128-token vocabulary; generation keeps a per-layer KV cache.
"""
from __future__ import annotations

import logging
import math
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd import ops

logger = logging.getLogger(__name__)

@dataclass
class T5Config:
    vocab_size: int = 32128
    d_model: int = 768
    d_kv: int = 64
    d_ff: int = 3072
    num_layers: int = 12
    num_decoder_layers: int = 12
    num_heads: int = 12
    relative_attention_num_buckets: int = 32
    relative_attention_max_distance: int = 128
    dropout_rate: float = 0.1
    layer_norm_epsilon: float = 1e-6
    gated_gelu: bool = False          # T5 v1.1 feed-forward
    pad_token_id: int = 0
    decoder_start_token_id: int = 0
    eos_token_id: int = 1

    @classmethod
    def small(cls, **kw):
        return cls(d_model=512, d_ff=2048, num_layers=6, num_decoder_layers=6, num_heads=8, **kw)

    @classmethod
    def base(cls, **kw):
        return cls(**kw)

    @classmethod
    def large(cls, **kw):
        return cls(d_model=1024, d_ff=4096, num_layers=24, num_decoder_layers=24, num_heads=16, **kw)

    @classmethod
    def tiny(cls, **kw):
        base = dict(vocab_size=64, d_model=32, d_kv=8, d_ff=64, num_layers=2, num_decoder_layers=2, num_heads=4,
                    relative_attention_num_buckets=8, relative_attention_max_distance=16, dropout_rate=0.0)
        base.update(kw)
        return cls(**base)


def relative_position_bucket(rel: torch.Tensor, bidirectional: bool, num_buckets: int, max_distance: int):
    """T5 bucketing of (key - query) offsets: exact buckets for small offsets, log-spaced
    buckets up to ``max_distance``, one shared bucket beyond."""
    ret = torch.zeros_like(rel)
    if bidirectional:
        num_buckets //= 2
        ret = ret + (rel > 0).long() * num_buckets
        n = rel.abs()
    else:
        n = (-rel).clamp(min=0)
    max_exact = num_buckets // 2
    small = n < max_exact
    large = max_exact + (torch.log(n.float().clamp(min=1) / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).long()
    large = large.clamp(max=num_buckets - 1)
    return ret + torch.where(small, n, large)


class T5Norm(nn.Module):
    def __init__(self, d, eps, device=None, dtype=None):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d, device=device, dtype=dtype))
        self.eps = eps

    def forward(self, x, residual=None):
        return ops.layer_norm(x, self.weight, None, eps=self.eps, residual=residual, rms=True)


class T5Attention(nn.Module):
    def __init__(self, cfg: T5Config, relative_bias: bool, causal: bool, device=None, dtype=None):
        super().__init__()
        inner = cfg.num_heads * cfg.d_kv
        kw = dict(bias=False, device=device, dtype=dtype)
        self.q, self.k, self.v = nn.Linear(cfg.d_model, inner, **kw), nn.Linear(cfg.d_model, inner, **kw), \
            nn.Linear(cfg.d_model, inner, **kw)
        self.o = nn.Linear(inner, cfg.d_model, **kw)
        self.h, self.dk = cfg.num_heads, cfg.d_kv
        self.causal = causal
        self.cfg = cfg
        self.rel = nn.Embedding(cfg.relative_attention_num_buckets, cfg.num_heads, device=device, dtype=dtype) \
            if relative_bias else None

    def relative_vector(self, sq: int, sk: int, device, offset: int = 0):
        """Per-head bias for every (key - query) offset: ``relvec [H, sq + sk - 1]`` with
        ``score(q, k) += relvec[h, k - q + rel_base]``, ``rel_base = sq - 1``; query
        positions start at ``offset`` (decoding with a KV cache)."""
        rel_base = sq - 1
        rel = torch.arange(sq + sk - 1, device=device) - rel_base - offset
        bucket = relative_position_bucket(rel, not self.causal, self.cfg.relative_attention_num_buckets,
                                          self.cfg.relative_attention_max_distance)
        return self.rel(bucket).t().float(), rel_base

    @staticmethod
    def full_bias(relvec, rel_base, sq, sk, causal_offset=None, key_bias=None):
        """Materialised [B|1, H, sq, sk] additive bias (the SDPA path)."""
        dev = relvec.device
        idx = torch.arange(sk, device=dev)[None, :] - torch.arange(sq, device=dev)[:, None] + rel_base
        bias = relvec[:, idx][None]
        if causal_offset is not None:
            allowed = torch.ones(sq, sk, dtype=torch.bool, device=dev).tril(causal_offset)
            bias = bias.masked_fill(~allowed, float("-inf"))
        if key_bias is not None:
            bias = bias + key_bias[:, None, None, :]
        return bias

    def _split(self, x):
        B, S, _ = x.shape
        return x.view(B, S, self.h, self.dk)

    def forward(self, x, kv=None, rel=None, key_bias=None, cache=None, offset: int = 0):
        """``kv``: encoder states for cross-attention; ``rel``: (relvec, rel_base) of the stack;
        ``key_bias`` [B, Sk] additive key mask; ``cache``: (k, v) of earlier decoder steps."""
        from cloudtik_amd import ops
        B, S, _ = x.shape
        q = self._split(self.q(x))                                    # [B, S, H, D]
        src = x if kv is None else kv
        if kv is not None and cache is not None:
            k, v = cache                                              # cross-attention K/V computed once
        else:
            k, v = self._split(self.k(src)), self._split(self.v(src))
            if cache is not None:
                k, v = torch.cat([cache[0], k], 1), torch.cat([cache[1], v], 1)
        Sk = k.shape[1]
        grad = torch.is_grad_enabled() and self.training
        kernel_ok = q.is_cuda and q.dtype == torch.bfloat16 and self.dk == 64
        # causal masking in the kernel is top-left aligned: exact for prefill (offset 0) and for
        # single-token decode steps (every cached key is visible)
        causal = self.causal and S > 1
        if rel is not None and kernel_ok and not grad and (offset == 0 or not causal):
            relvec, rel_base = rel
            o = ops.attention_relbias(q, k, v, relvec, rel_base, key_bias, scale=1.0, causal=causal)
        elif rel is None and kernel_ok and not (self.training and self.cfg.dropout_rate):
            o = ops.attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), key_bias=key_bias,
                              scale=1.0, causal=causal).transpose(1, 2)          # T5 folds the scale into init
        else:
            bias = None
            if rel is not None:
                bias = self.full_bias(rel[0], rel[1], S, Sk, offset if causal else None, key_bias)
            elif key_bias is not None:
                bias = key_bias[:, None, None, :]
            o = F.scaled_dot_product_attention(
                q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                attn_mask=bias.to(q.dtype) if bias is not None else None,
                dropout_p=self.cfg.dropout_rate if self.training else 0.0,
                is_causal=causal and bias is None, scale=1.0).transpose(1, 2)
        return self.o(o.reshape(B, S, -1)), (k, v)


class T5FF(nn.Module):
    def __init__(self, cfg: T5Config, device=None, dtype=None):
        super().__init__()
        kw = dict(bias=False, device=device, dtype=dtype)
        self.gated = cfg.gated_gelu
        self.wi = nn.Linear(cfg.d_model, cfg.d_ff, **kw)
        if self.gated:
            self.wi_1 = nn.Linear(cfg.d_model, cfg.d_ff, **kw)
        self.wo = nn.Linear(cfg.d_ff, cfg.d_model, **kw)
        self.p = cfg.dropout_rate

    def forward(self, x):
        h = F.gelu(self.wi(x), approximate="tanh") * self.wi_1(x) if self.gated else F.relu(self.wi(x))
        if self.training and self.p:
            h = F.dropout(h, self.p)
        return self.wo(h)


class T5Block(nn.Module):
    def __init__(self, cfg: T5Config, decoder: bool, relative_bias: bool, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.ln_sa = T5Norm(cfg.d_model, cfg.layer_norm_epsilon, **kw)
        self.sa = T5Attention(cfg, relative_bias, causal=decoder, **kw)
        self.decoder = decoder
        if decoder:
            self.ln_ca = T5Norm(cfg.d_model, cfg.layer_norm_epsilon, **kw)
            self.ca = T5Attention(cfg, False, causal=False, **kw)
        self.ln_ff = T5Norm(cfg.d_model, cfg.layer_norm_epsilon, **kw)
        self.ff = T5FF(cfg, **kw)
        self.p = cfg.dropout_rate

    def _drop(self, x):
        return F.dropout(x, self.p) if (self.training and self.p) else x

    def forward(self, x, rel, key_bias=None, enc=None, enc_bias=None, cache=None, offset: int = 0):
        new_cache = {}
        h, new_cache["self"] = self.sa(self.ln_sa(x), rel=rel, key_bias=key_bias,
                                       cache=cache.get("self") if cache else None, offset=offset)
        x = x + self._drop(h)
        if self.decoder:
            h, new_cache["cross"] = self.ca(self.ln_ca(x), kv=enc, key_bias=enc_bias,
                                            cache=cache.get("cross") if cache else None)
            x = x + self._drop(h)
        x = x + self._drop(self.ff(self.ln_ff(x)))
        return x, new_cache


class T5Stack(nn.Module):
    def __init__(self, cfg: T5Config, decoder: bool, embed: nn.Embedding, device=None, dtype=None):
        super().__init__()
        n = cfg.num_decoder_layers if decoder else cfg.num_layers
        self.embed = embed
        self.blocks = nn.ModuleList([T5Block(cfg, decoder, i == 0, device, dtype) for i in range(n)])
        self.final = T5Norm(cfg.d_model, cfg.layer_norm_epsilon, device, dtype)
        self.decoder = decoder
        self.p = cfg.dropout_rate

    def forward(self, ids, mask=None, enc=None, enc_mask=None, caches=None, offset: int = 0):
        x = self.embed(ids)
        if self.training and self.p:
            x = F.dropout(x, self.p)
        B, S = ids.shape
        sk = S + offset
        rel = self.blocks[0].sa.relative_vector(S, sk, ids.device, offset)
        key_bias = (1.0 - mask.float()) * -1e9 if mask is not None else None
        enc_bias = (1.0 - enc_mask.float()) * -1e9 if enc_mask is not None else None
        new_caches = []
        for i, blk in enumerate(self.blocks):
            x, c = blk(x, rel, key_bias, enc, enc_bias, caches[i] if caches else None, offset)
            new_caches.append(c)
        x = self.final(x)
        if self.training and self.p:
            x = F.dropout(x, self.p)
        return x, new_caches


class T5ForConditionalGeneration(nn.Module):
    def __init__(self, cfg: T5Config = None, device=None, dtype=torch.bfloat16):
        super().__init__()
        cfg = cfg or T5Config()
        self.cfg = cfg
        self.shared = nn.Embedding(cfg.vocab_size, cfg.d_model, device=device, dtype=dtype)
        nn.init.normal_(self.shared.weight, std=1.0)
        self.encoder = T5Stack(cfg, False, self.shared, device, dtype)
        self.decoder = T5Stack(cfg, True, self.shared, device, dtype)
        self.dtype = dtype

    def _shift_right(self, labels):
        start = torch.full_like(labels[:, :1], self.cfg.decoder_start_token_id)
        ids = torch.cat([start, labels[:, :-1]], 1)
        return ids.masked_fill(ids == -100, self.cfg.pad_token_id)

    def forward(self, input_ids, labels, attention_mask=None, decoder_input_ids=None):
        """Training: mean token cross-entropy (tied, d_model^-0.5-scaled output head)."""
        enc, _ = self.encoder(input_ids, attention_mask)
        dec_ids = decoder_input_ids if decoder_input_ids is not None else self._shift_right(labels)
        dec, _ = self.decoder(dec_ids, enc=enc, enc_mask=attention_mask)
        x = (dec * (self.cfg.d_model ** -0.5)).reshape(-1, self.cfg.d_model)
        return ops.cross_entropy_fused(x, self.shared.weight, None, labels.reshape(-1), ignore_index=-100)

    def logits(self, dec):
        return F.linear(dec * (self.cfg.d_model ** -0.5), self.shared.weight)

    @torch.no_grad()
    def generate(self, input_ids, attention_mask=None, max_new_tokens: int = 32,
                 use_graph: Optional[bool] = None) -> torch.Tensor:
        """Greedy decoding with a KV cache (self-attention K/V grow; cross K/V computed once).

        On the GPU the decode step is captured once into a HIP graph over a static KV cache
        of ``max_new_tokens`` slots and replayed per token (``_generate_graph``): a decode step
        is ~15 small kernels per layer, so launch overhead, not math, bounds eager decoding."""
        if use_graph is None:
            use_graph = input_ids.is_cuda and os.environ.get("CLOUDTIK_AMD_T5_GRAPH", "1") == "1"
        if use_graph and input_ids.is_cuda:
            try:
                return self._generate_graph(input_ids, attention_mask, max_new_tokens)
            except RuntimeError as e:          # capture unsupported by some op: eager fallback
                logger.warning("T5 graph decoding unavailable (%s); decoding eagerly", e)
        enc, _ = self.encoder(input_ids, attention_mask)
        B = input_ids.shape[0]
        cur = torch.full((B, 1), self.cfg.decoder_start_token_id, dtype=torch.long, device=input_ids.device)
        out, caches = [], None
        done = torch.zeros(B, dtype=torch.bool, device=input_ids.device)
        for step in range(max_new_tokens):
            dec, caches = self.decoder(cur, enc=enc, enc_mask=attention_mask, caches=caches, offset=step)
            nxt = self.logits(dec[:, -1]).float().argmax(-1)
            nxt = torch.where(done, torch.full_like(nxt, self.cfg.pad_token_id), nxt)
            out.append(nxt)
            done |= nxt == self.cfg.eos_token_id
            cur = nxt[:, None]
        return torch.stack(out, 1)

    def _generate_graph(self, input_ids, attention_mask, max_new: int) -> torch.Tensor:
        """Graph-replayed greedy decoding.  The captured graph and its static buffers are cached
        per (batch, source length, steps, masked): a later call only runs the encoder, copies the
        cross-attention K/V and the source mask into the static buffers and replays."""
        cfg = self.cfg
        dev = input_ids.device
        B, S, T = input_ids.shape[0], input_ids.shape[1], max_new
        dec = self.decoder
        enc, _ = self.encoder(input_ids, attention_mask)
        key = (B, S, T, attention_mask is not None, str(dev))
        cache = getattr(self, "_graphs", None)
        if cache is None:
            cache = self._graphs = {}
        st = cache.get(key)
        if st is None:
            st = cache[key] = self._capture_decode(B, S, T, enc.dtype, dev, attention_mask is not None)
        for i, b in enumerate(dec.blocks):
            st["cross"][i][0].copy_(b.ca._split(b.ca.k(enc)))
            st["cross"][i][1].copy_(b.ca._split(b.ca.v(enc)))
        if attention_mask is not None:
            st["enc_bias"].copy_((1.0 - attention_mask.float()) * -1e9)
        st["reset"]()
        for _ in range(T):
            st["graph"].replay()
        return st["out"].clone()

    def _capture_decode(self, B, S, T, dtype, dev, masked: bool):
        cfg = self.cfg
        H, D = cfg.num_heads, cfg.d_kv
        dec = self.decoder
        kc = [torch.zeros(B, T, H, D, dtype=dtype, device=dev) for _ in dec.blocks]
        vc = [torch.zeros(B, T, H, D, dtype=dtype, device=dev) for _ in dec.blocks]
        cross = [(torch.zeros(B, S, H, D, dtype=dtype, device=dev), torch.zeros(B, S, H, D, dtype=dtype, device=dev))
                 for _ in dec.blocks]
        enc_bias = torch.zeros(B, S, device=dev) if masked else None
        cur = torch.full((B, 1), cfg.decoder_start_token_id, dtype=torch.long, device=dev)
        pos = torch.zeros(1, dtype=torch.long, device=dev)
        out = torch.full((B, T), cfg.pad_token_id, dtype=torch.long, device=dev)
        done = torch.zeros(B, dtype=torch.bool, device=dev)
        slots = torch.arange(T, device=dev)
        pad = torch.full((B,), cfg.pad_token_id, dtype=torch.long, device=dev)
        sa0 = dec.blocks[0].sa

        def step():
            x = dec.embed(cur)
            bucket = relative_position_bucket(slots - pos, False, cfg.relative_attention_num_buckets,
                                              cfg.relative_attention_max_distance)
            relvec = sa0.rel(bucket).t().float().contiguous()              # query at `pos`, keys 0..T-1
            key_bias = torch.where(slots <= pos, 0.0, -1e9).float()[None].expand(B, T).contiguous()
            for i, blk in enumerate(dec.blocks):
                h = blk.ln_sa(x)
                a = blk.sa
                q, k, v = a._split(a.q(h)), a._split(a.k(h)), a._split(a.v(h))
                kc[i].index_copy_(1, pos, k)
                vc[i].index_copy_(1, pos, v)
                o = ops.attention_relbias(q, kc[i], vc[i], relvec, 0, key_bias, scale=1.0, causal=False)
                x = x + a.o(o.reshape(B, 1, -1))
                h = blk.ln_ca(x)
                c = blk.ca
                q = c._split(c.q(h))
                o = ops.attention(q.transpose(1, 2), cross[i][0].transpose(1, 2), cross[i][1].transpose(1, 2),
                                  key_bias=enc_bias, scale=1.0).transpose(1, 2)
                x = x + c.o(o.reshape(B, 1, -1))
                x = x + blk.ff(blk.ln_ff(x))
            x = dec.final(x)
            nxt = self.logits(x[:, -1]).float().argmax(-1)
            nxt = torch.where(done, pad, nxt)
            out.index_copy_(1, pos, nxt[:, None])
            done.logical_or_(nxt == cfg.eos_token_id)
            cur.copy_(nxt[:, None])
            pos.add_(1)

        def reset():
            cur.fill_(cfg.decoder_start_token_id)
            pos.zero_()
            out.fill_(cfg.pad_token_id)
            done.zero_()

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):          # warm up (lazy inits, library handles) off the capture
            step()
        torch.cuda.current_stream().wait_stream(side)
        reset()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        return {"graph": graph, "cross": cross, "enc_bias": enc_bias, "out": out, "reset": reset}
