"""Side-stream weight gradients: identical gradients to the serial schedule (BERT-base shape)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
from cloudtik_amd import ops
import importlib
L = importlib.import_module("cloudtik_amd.ops.linear")
from cloudtik_amd.models.bert import BertConfig, BertForPreTraining, synthetic_pretraining_batch
from cloudtik_amd.train.optim import FlatParamSpace

dev = torch.device("cuda")
grads = []
for side in (False, True):
    ops.manual_seed(5)
    torch.manual_seed(5)
    cfg = BertConfig.base()
    cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    m = BertForPreTraining(cfg, device=dev, dtype=torch.bfloat16)
    L.use_wgrad_side_stream(m, side)
    named = list(m.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    batch = synthetic_pretraining_batch(cfg, 32, 128, 20, device=dev, generator=torch.Generator().manual_seed(1))
    for _ in range(2):
        space.grad.zero_()
        m(**batch).backward()
        L.sync_grad_stream()
    torch.cuda.synchronize()
    grads.append(space.grad.float().clone())
d = (grads[0] - grads[1]).abs().max().item()
print(f"max |grad serial - grad side-stream| = {d}", flush=True)
assert d == 0.0, d
