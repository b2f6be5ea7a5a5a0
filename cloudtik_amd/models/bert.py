"""BERT (pretraining: masked-LM + next-sentence) built on the cloudtik_amd op library.

Functional parity target: the HF ``BertForPreTraining`` the reference instantiates from a
config for its BERT-large MLPerf pretraining (applications/ai/quickstart/models/
language_modeling/pytorch/bert_large/training/run_pretrain_mlperf.py:449-471), with
``dense_seq_output`` (masked-LM head evaluated only at masked positions, :462, :578-590).

MI355X-first structure of one encoder layer (bf16 activations/weights, fp32 statistics):

    qkv  = x @ Wqkv^T + bqkv                 one packed hipBLASLt GEMM (bias epilogue)
    ctx  = attention_packed(qkv)             HIP MFMA flash attention, reads Q/K/V by stride
    a    = ctx @ Wo^T                        bias-free GEMM
    x1   = LN(x + dropout(a + bo))           ONE HIP kernel (bias + dropout + residual + LN)
    z    = x1 @ W1^T                         bias-free GEMM
    h    = gelu(z + b1)                      HIP bias-GELU (keeps z for backward)
    f    = h @ W2^T                          bias-free GEMM
    x2   = LN(x1 + dropout(f + b2))          ONE HIP kernel

so every bias gradient is folded into a LayerNorm / bias-GELU backward kernel and there is
no permute/contiguous copy anywhere in the layer.  The vocabulary is padded to a multiple
of 256 rows (aligned 16-byte vector access in the fused cross-entropy kernel, and whole
256-row tiles for the decoder's weight-gradient GEMM); padded rows never receive tokens and
are masked out of the softmax.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, asdict

import torch
import torch.nn as nn
import torch.nn.functional as F

from cloudtik_amd.ops.linear import use_wgrad_side_stream
from cloudtik_amd import ops


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 1024
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 4096
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02
    pad_vocab_multiple: int = 256
    dense_seq_output: bool = True

    @property
    def padded_vocab(self) -> int:
        m = self.pad_vocab_multiple
        return ((self.vocab_size + m - 1) // m) * m

    @classmethod
    def large(cls, **kw):
        return cls(**kw)

    @classmethod
    def base(cls, **kw):
        d = dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072)
        d.update(kw)
        return cls(**d)

    @classmethod
    def tiny(cls, **kw):
        d = dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                 intermediate_size=512, max_position_embeddings=128)
        d.update(kw)
        return cls(**d)

    @classmethod
    def from_dict(cls, d):
        keys = set(cls.__dataclass_fields__)
        return cls(**{k: v for k, v in d.items() if k in keys})

    def to_dict(self):
        return asdict(self)


def _param(*shape, std=None, fill=None, device=None, dtype=None):
    t = torch.empty(*shape, device=device, dtype=torch.float32)
    if std is not None:
        nn.init.normal_(t, 0.0, std)
    else:
        t.fill_(fill)
    return nn.Parameter(t.to(dtype))


class BertLayer(nn.Module):
    def __init__(self, cfg: BertConfig, device=None, dtype=None):
        super().__init__()
        H, I = cfg.hidden_size, cfg.intermediate_size
        std = cfg.initializer_range
        kw = dict(device=device, dtype=dtype)
        self.cfg = cfg
        self.qkv_weight = _param(3 * H, H, std=std, **kw)
        self.qkv_bias = _param(3 * H, fill=0.0, **kw)
        self.out_weight = _param(H, H, std=std, **kw)
        self.out_bias = _param(H, fill=0.0, **kw)
        self.ln1_weight = _param(H, fill=1.0, **kw)
        self.ln1_bias = _param(H, fill=0.0, **kw)
        self.ffn1_weight = _param(I, H, std=std, **kw)
        self.ffn1_bias = _param(I, fill=0.0, **kw)
        self.ffn2_weight = _param(H, I, std=std, **kw)
        self.ffn2_bias = _param(H, fill=0.0, **kw)
        self.ln2_weight = _param(H, fill=1.0, **kw)
        self.ln2_bias = _param(H, fill=0.0, **kw)

    def forward(self, x, key_bias):
        cfg = self.cfg
        tr = self.training
        from cloudtik_amd.ops import transformer as T
        if T.blocks_supported(x, cfg.hidden_size, cfg.num_attention_heads):
            # hand-scheduled blocks: one autograd node each, fused residual/bias/wgrad grads
            x1 = T.attention_block(x, self.qkv_weight, self.qkv_bias, self.out_weight, self.out_bias,
                                   self.ln1_weight, self.ln1_bias, key_bias, cfg.num_attention_heads,
                                   cfg.attention_probs_dropout_prob, cfg.hidden_dropout_prob,
                                   cfg.layer_norm_eps, tr)
            return T.ffn_block(x1, self.ffn1_weight, self.ffn1_bias, self.ffn2_weight, self.ffn2_bias,
                               self.ln2_weight, self.ln2_bias, cfg.hidden_dropout_prob,
                               cfg.layer_norm_eps, tr)
        qkv = ops.linear(x, self.qkv_weight, self.qkv_bias)
        ctx = ops.attention_packed(qkv, cfg.num_attention_heads, key_bias,
                                   p=cfg.attention_probs_dropout_prob, training=tr)
        a = ops.linear(ctx, self.out_weight)
        x1 = ops.layer_norm(a, self.ln1_weight, self.ln1_bias, cfg.layer_norm_eps,
                            bias=self.out_bias, residual=x, p=cfg.hidden_dropout_prob, training=tr)
        z = ops.linear(x1, self.ffn1_weight)
        h = ops.bias_gelu(z, self.ffn1_bias)
        f = ops.linear(h, self.ffn2_weight)
        return ops.layer_norm(f, self.ln2_weight, self.ln2_bias, cfg.layer_norm_eps,
                              bias=self.ffn2_bias, residual=x1, p=cfg.hidden_dropout_prob, training=tr)


class BertModel(nn.Module):
    def __init__(self, cfg: BertConfig, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        H = cfg.hidden_size
        kw = dict(device=device, dtype=dtype)
        std = cfg.initializer_range
        self.word_embeddings = _param(cfg.padded_vocab, H, std=std, **kw)
        self.position_embeddings = _param(cfg.max_position_embeddings, H, std=std, **kw)
        self.token_type_embeddings = _param(cfg.type_vocab_size, H, std=std, **kw)
        self.emb_ln_weight = _param(H, fill=1.0, **kw)
        self.emb_ln_bias = _param(H, fill=0.0, **kw)
        self.layers = nn.ModuleList([BertLayer(cfg, **kw) for _ in range(cfg.num_hidden_layers)])
        self.pooler_weight = _param(H, H, std=std, **kw)
        self.pooler_bias = _param(H, fill=0.0, **kw)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None):
        cfg = self.cfg
        emb = ops.embedding3(input_ids, token_type_ids, self.word_embeddings,
                             self.position_embeddings, self.token_type_embeddings)
        x = ops.layer_norm(emb, self.emb_ln_weight, self.emb_ln_bias, cfg.layer_norm_eps)
        x = ops.dropout(x, cfg.hidden_dropout_prob, self.training)
        key_bias = None
        if attention_mask is not None:
            key_bias = (1.0 - attention_mask.to(torch.float32)) * -10000.0
        for layer in self.layers:
            x = layer(x, key_bias)
        pooled = torch.tanh(F.linear(x[:, 0], self.pooler_weight, self.pooler_bias))
        return x, pooled


class BertForPreTraining(nn.Module):
    """Masked-LM + next-sentence-prediction heads; returns the summed loss."""

    def __init__(self, cfg: BertConfig, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.cfg = cfg
        H = cfg.hidden_size
        kw = dict(device=device, dtype=dtype)
        std = cfg.initializer_range
        self.bert = BertModel(cfg, **kw)
        self.mlm_dense_weight = _param(H, H, std=std, **kw)
        self.mlm_dense_bias = _param(H, fill=0.0, **kw)
        self.mlm_ln_weight = _param(H, fill=1.0, **kw)
        self.mlm_ln_bias = _param(H, fill=0.0, **kw)
        self.mlm_decoder_bias = _param(cfg.padded_vocab, fill=0.0, **kw)
        self.nsp_weight = _param(2, H, std=std, **kw)
        self.nsp_bias = _param(2, fill=0.0, **kw)
        # GEMM-bound backward: weight gradients in line, not on the side stream (the model's
        # own routing, the same at every world size; ops/linear.py use_wgrad_side_stream)
        use_wgrad_side_stream(self, False)

    def mlm_loss(self, seq, masked_lm_positions=None, masked_lm_ids=None, masked_lm_labels=None):
        cfg = self.cfg
        B, S, H = seq.shape
        if masked_lm_positions is not None:
            # static-shape gather of the masked slots (no host sync): [B, P] positions
            idx = masked_lm_positions + torch.arange(B, device=seq.device).unsqueeze(1) * S
            rows = seq.reshape(B * S, H).index_select(0, idx.reshape(-1))
            labels = masked_lm_ids.reshape(-1)
        else:
            rows = seq.reshape(B * S, H)
            labels = masked_lm_labels.reshape(-1)
        t = ops.linear(rows, self.mlm_dense_weight)
        t = ops.bias_gelu(t, self.mlm_dense_bias)
        t = ops.layer_norm(t, self.mlm_ln_weight, self.mlm_ln_bias, cfg.layer_norm_eps)
        return ops.cross_entropy_fused(t, self.bert.word_embeddings, self.mlm_decoder_bias, labels,
                                       V=cfg.vocab_size, ignore_index=-100)

    def forward(self, input_ids, token_type_ids=None, attention_mask=None, masked_lm_positions=None,
                masked_lm_ids=None, masked_lm_labels=None, next_sentence_labels=None):
        seq, pooled = self.bert(input_ids, token_type_ids, attention_mask)
        loss = self.mlm_loss(seq, masked_lm_positions, masked_lm_ids, masked_lm_labels)
        if next_sentence_labels is not None:
            nsp_logits = F.linear(pooled, self.nsp_weight, self.nsp_bias)
            loss = loss + F.cross_entropy(nsp_logits.float(), next_sentence_labels.reshape(-1))
        return loss

    @staticmethod
    def no_decay(name: str) -> bool:
        """Parameters excluded from weight decay (reference: bias / LayerNorm, :495)."""
        return name.endswith("bias") or "ln" in name.split(".")[-1]


def synthetic_pretraining_batch(cfg: BertConfig, batch: int, seq_len: int = 128,
                                max_pred: int = 20, device=None, generator=None):
    """Random batch in the MLPerf HDF5 shard format (positions/ids per masked slot)."""
    g = generator
    ids = torch.randint(0, cfg.vocab_size, (batch, seq_len), generator=g)
    tt = torch.zeros(batch, seq_len, dtype=torch.long)
    tt[:, seq_len // 2:] = 1
    mask = torch.ones(batch, seq_len, dtype=torch.long)
    pos = torch.stack([torch.randperm(seq_len - 1, generator=g)[:max_pred] + 1 for _ in range(batch)])
    pos, _ = pos.sort(1)
    mids = torch.randint(0, cfg.vocab_size, (batch, max_pred), generator=g)
    nsp = torch.randint(0, 2, (batch,), generator=g)
    out = dict(input_ids=ids, token_type_ids=tt, attention_mask=mask, masked_lm_positions=pos,
               masked_lm_ids=mids, next_sentence_labels=nsp)
    if device is not None:
        out = {k: v.to(device, non_blocking=True) for k, v in out.items()}
    return out


def flops_per_sequence(cfg: BertConfig, seq_len: int, max_pred: int) -> float:
    """Training FLOPs (fwd + bwd = 3x fwd) of one sequence, GEMMs + attention."""
    H, I, L = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    per_tok_layer = 2 * (4 * H * H + 2 * H * I) + 4 * seq_len * H
    mlm = max_pred * 2 * (H * H + H * cfg.padded_vocab)
    return 3.0 * (L * seq_len * per_tok_layer + mlm)
