"""Stock PyTorch-ROCm baselines for the headline benchmark.

``bench.py --impl eager`` runs the SAME configurations as the native path, built only from
what a user gets out of the box -- so the JSON can report how much the custom stack buys:

* BERT-large: Hugging Face ``BertForPreTraining`` (the model the reference instantiates,
  run_pretrain_mlperf.py:449-471) with ``attn_implementation="sdpa"``, fp32 parameters under
  ``torch.autocast(bfloat16)``, ``DistributedDataParallel`` and the per-tensor LAMB below;
* ResNet-50: the v1.5 topology from ``nn.Conv2d`` / ``nn.BatchNorm2d`` / ``nn.ReLU``,
  channels_last, autocast bf16, DDP, ``torch.optim.SGD`` (foreach).

``ReferenceLAMB`` implements the reference's update rule
(applications/ai/quickstart/models/language_modeling/pytorch/bert_large/training/lamb.py:61-139):
no bias correction, ``adam_step = m / (sqrt(v) + eps)``, weight decay added to the step and
a trust ratio ``||w|| / ||step||`` only for tensors whose group has weight_decay != 0, bf16
parameters stepped through an fp32 master copy.  The zero-norm guard is a ``torch.where``
instead of the reference's host-side comparison (same values, no device->host sync).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class ReferenceLAMB(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            b1, b2 = group["betas"]
            wd, lr, eps = group["weight_decay"], group["lr"], group["eps"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                low = p.dtype != torch.float32
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32)
                    if low:
                        st["master"] = p.detach().float().clone()
                st["step"] += 1
                g = p.grad.float()
                w = st["master"] if low else p
                m, v = st["exp_avg"], st["exp_avg_sq"]
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                upd = m / (v.sqrt() + eps)
                if wd != 0:
                    upd.add_(w, alpha=wd)
                    wn = w.norm()
                    un = upd.norm()
                    ratio = torch.where((wn > 0) & (un > 0), wn / un, torch.ones_like(wn))
                    w.sub_(upd * (lr * ratio))
                else:
                    w.sub_(upd, alpha=lr)
                if low:
                    p.copy_(w)
        return loss


def lamb_param_groups(model: nn.Module, weight_decay: float):
    """Reference grouping (run_pretrain_mlperf.py:491-497): no decay on bias / LayerNorm."""
    decay, nodecay = [], []
    for n, p in model.named_parameters():
        (nodecay if ("bias" in n or "LayerNorm" in n or "gamma" in n or "beta" in n) else decay).append(p)
    return [{"params": decay, "weight_decay": weight_decay}, {"params": nodecay, "weight_decay": 0.0}]


def hf_bert_config(large: bool = True, **kw):
    from transformers import BertConfig
    d = dict(vocab_size=30522, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
             intermediate_size=4096, hidden_act="gelu", max_position_embeddings=512, type_vocab_size=2,
             layer_norm_eps=1e-12, initializer_range=0.02)
    if not large:
        d.update(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072)
    d.update(kw)
    return BertConfig(**d)


def build_hf_bert(hf_cfg, device):
    from transformers import BertForPreTraining
    torch.manual_seed(1234)
    try:
        model = BertForPreTraining._from_config(hf_cfg, attn_implementation="sdpa")
    except TypeError:  # older transformers
        model = BertForPreTraining(hf_cfg)
    return model.to(device)


def dense_mlm_labels(batch, seq_len):
    """MLPerf slot format (positions / ids) -> HF's [B, S] label tensor (-100 elsewhere)."""
    pos, ids = batch["masked_lm_positions"], batch["masked_lm_ids"]
    B = pos.shape[0]
    lab = torch.full((B, seq_len), -100, dtype=torch.long, device=pos.device)
    lab.scatter_(1, pos, ids)
    return lab


# ---------------------------------------------------------------- stock ResNet-50 (v1.5)
class _Bottleneck(nn.Module):
    def __init__(self, cin, width, stride, down):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.relu = nn.ReLU(inplace=True)
        self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout)) \
            if down else None

    def forward(self, x):
        idt = self.down(x) if self.down is not None else x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        return self.relu(self.bn3(self.conv3(out)) + idt)


class StockResNet50(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                                  nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], 64
        for i, (n, w) in enumerate(zip((3, 4, 6, 3), (64, 128, 256, 512))):
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(_Bottleneck(cin, w, stride, j == 0))
                cin = w * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))
