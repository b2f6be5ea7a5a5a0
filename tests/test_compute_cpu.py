"""CPU checks of the compute stack's torch paths (the HIP paths are pinned against the same
references in test_ops_gpu.py).  Reference test strategy: the AI runtime's examples are
smoke-run end to end."""
import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from cloudtik_amd.ops import reference as R


def test_hash_dropout_mask_deterministic_and_rate():
    m1 = R.dropout_keep_mask(1 << 16, 0.1, seed=7, offset=0)
    m2 = R.dropout_keep_mask(1 << 16, 0.1, seed=7, offset=0)
    m3 = R.dropout_keep_mask(1 << 16, 0.1, seed=7, offset=1 << 16)
    assert torch.equal(m1, m2) and not torch.equal(m1, m3)
    assert abs(1 - m1.float().mean().item() - 0.1) < 0.01


def test_hash_dropout_mask_statistics():
    """Per-lane drop rates, independence of the two elements sharing one hash, and no
    correlation between the streams of consecutive offsets (steps)."""
    n, p = 1 << 20, 0.1
    d = ~R.dropout_keep_mask(n, p, seed=11, offset=0)
    lanes = d.view(-1, 8).float().mean(0)
    assert torch.all((lanes - p).abs() < 0.004), lanes
    pairs = d.view(-1, 2)
    both = (pairs[:, 0] & pairs[:, 1]).float().mean().item()
    assert abs(both - p * p) < 0.002, both
    d2 = ~R.dropout_keep_mask(n, p, seed=11, offset=n)
    assert abs((d & d2).float().mean().item() - p * p) < 0.002
    # neighbouring 8-element vectors are independent too
    v = d.view(-1, 8).any(1).float()
    assert abs((v[1:] * v[:-1]).mean().item() - v.mean().item() ** 2) < 0.005


def test_attention_dropout_mask_rate():
    k = R.attn_dropout_keep(2, 2, 64, 64, 0.2, seed=3, offset=0)
    assert abs(1 - k.float().mean().item() - 0.2) < 0.02


def test_reference_layer_norm_matches_torch():
    x = torch.randn(8, 64)
    g, b = torch.rand(64), torch.randn(64)
    y = R.layer_norm(x, g, b, eps=1e-5)
    y = y[0] if isinstance(y, tuple) else y
    torch.testing.assert_close(y, torch.nn.functional.layer_norm(x, (64,), g, b, 1e-5), atol=1e-5, rtol=1e-5)


def test_reference_attention_matches_sdpa():
    q, k, v = (torch.randn(2, 4, 16, 8) for _ in range(3))
    out = R.attention(q, k, v)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    out = R.attention(q, k, v, causal=True)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)


def test_functional_ops_cpu_autograd():
    from cloudtik_amd import ops
    x = torch.randn(4, 32, requires_grad=True)
    g = torch.ones(32, requires_grad=True)
    b = torch.zeros(32, requires_grad=True)
    y = ops.layer_norm(x, g, b, eps=1e-5)
    y = y[0] if isinstance(y, tuple) else y
    y.sum().backward()
    assert x.grad is not None and g.grad is not None
    z = torch.randn(4, 32, requires_grad=True)
    ops.bias_gelu(z, torch.zeros(32)).sum().backward()
    assert z.grad is not None


def test_bert_tiny_cpu_train_step_loss_decreases():
    from cloudtik_amd.models.bert import BertConfig, BertForPreTraining, synthetic_pretraining_batch
    from cloudtik_amd.train.optim import FlatParamSpace, FusedLAMB
    torch.manual_seed(0)
    cfg = BertConfig.tiny()
    cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    model = BertForPreTraining(cfg, device="cpu", dtype=torch.float32)
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedLAMB(space, lr=1e-2, weight_decay=0.01, no_decay=BertForPreTraining.no_decay)
    batch = synthetic_pretraining_batch(cfg, 4, 32, 5, device="cpu",
                                        generator=torch.Generator().manual_seed(1))
    losses = []
    for _ in range(6):
        loss = model(**batch)
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    assert all(math.isfinite(l) for l in losses)
    assert losses[-1] < losses[0]


def _ref_adamw(p, g, m, v, lr, b1, b2, eps, wd, step):
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    mh = m / (1 - b1 ** step)
    vh = v / (1 - b2 ** step)
    p.mul_(1 - lr * wd).sub_(lr * mh / (vh.sqrt() + eps))


def test_fused_adamw_cpu_matches_reference():
    from cloudtik_amd.train.optim import FlatParamSpace, FusedAdam
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(37)), torch.nn.Parameter(torch.randn(5, 3))]
    ref = [p.detach().clone() for p in params]
    space = FlatParamSpace(params, names=["a", "b"])
    opt = FusedAdam(space, lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.1, space=space)
    ms = [torch.zeros_like(r) for r in ref]
    vs = [torch.zeros_like(r) for r in ref]
    for step in range(1, 4):
        grads = [torch.randn_like(r) for r in ref]
        order = [id(q) for q in space.params]   # the flat space may reorder parameters
        for p, g in zip(params, grads):
            i = order.index(id(p))
            o, n = space.offsets[i], space.numels[i]
            space.grad[o:o + n].copy_(g.reshape(-1))
        opt.step()
        for r, g, m, v in zip(ref, grads, ms, vs):
            _ref_adamw(r, g, m, v, 1e-2, 0.9, 0.99, 1e-8, 0.1, step)
    for p, r in zip(params, ref):
        torch.testing.assert_close(p.detach().float(), r, atol=1e-5, rtol=1e-4)


def test_fused_sgd_cpu_momentum():
    from cloudtik_amd.train.optim import FlatParamSpace, FusedSGD
    p = torch.nn.Parameter(torch.ones(8))
    space = FlatParamSpace([p], names=["w"])
    opt = FusedSGD(space, lr=0.1, momentum=0.9, weight_decay=0.0, space=space)
    ref = torch.nn.Parameter(torch.ones(8))
    ropt = torch.optim.SGD([ref], lr=0.1, momentum=0.9)
    for _ in range(3):
        space.grad.fill_(0.5)
        opt.step()
        ref.grad = torch.full((8,), 0.5)
        ropt.step()
    torch.testing.assert_close(p.detach().float(), ref.detach(), atol=1e-6, rtol=1e-6)


def test_lr_schedulers():
    from cloudtik_amd.train.lr_scheduler import (LinearWarmUpScheduler, LinearWarmupPolyDecayScheduler,
                                                 StepDecayScheduler)
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    s = LinearWarmupPolyDecayScheduler(opt, start_warmup_steps=0, warmup_steps=10, total_steps=100,
                                       end_learning_rate=0.0, degree=1.0)
    lrs = []
    for _ in range(100):
        s.step()
        lrs.append(opt.param_groups[0]["lr"])
    assert lrs[0] < lrs[9] and lrs[-1] < lrs[50] < lrs[10] + 1e-9
    opt2 = torch.optim.SGD([p], lr=1.0)
    LinearWarmUpScheduler(opt2, warmup=0.1, total_steps=10).step()
    opt3 = torch.optim.SGD([p], lr=1.0)
    s3 = StepDecayScheduler(opt3, step_size=2, gamma=0.5)
    for _ in range(5):
        s3.step()
    assert opt3.param_groups[0]["lr"] < 1.0


def test_resnet_small_cpu_step():
    from cloudtik_amd.models.resnet import resnet18_like_small
    m = resnet18_like_small(num_classes=10)
    x = torch.randn(2, 3, 32, 32).contiguous(memory_format=torch.channels_last)
    out = m(x)
    assert out.shape == (2, 10)
    out.float().logsumexp(-1).sum().backward()
    assert any(p.grad is not None for p in m.parameters())


# ---------------------------------------------------------------------- multi-process gloo
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ddp_worker(rank, world, port, out):
    import torch.distributed as dist
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FlatParamSpace, FusedSGD
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different init per rank -> broadcast must fix it
    model = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedSGD(space, lr=0.1, momentum=0.0, space=space)
    broadcast_flat_params(space)
    ddp = GradBucketer(space, bucket_mb=0.0005)  # tiny buckets -> several buckets
    opt.grad_scale = ddp.grad_scale
    g = torch.Generator().manual_seed(rank)
    x, y = torch.randn(8, 16, generator=g), torch.randint(0, 4, (8,), generator=g)
    loss = torch.nn.functional.cross_entropy(model(x), y)
    loss.backward()
    ddp.finish()
    out[rank] = (space.grad.clone() * ddp.grad_scale, len(ddp.buckets))
    opt.step()
    flat = torch.cat([p.detach().reshape(-1) for _, p in named])
    out[rank] = out[rank] + (flat,)
    dist.destroy_process_group()


def test_gradbucketer_two_ranks_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        procs = [ctx.Process(target=_ddp_worker, args=(r, world, port, out)) for r in range(world)]
        [p.start() for p in procs]
        [p.join(120) for p in procs]
        assert all(p.exitcode == 0 for p in procs)
        g0, nb, w0 = out[0]
        g1, _, w1 = out[1]
    assert nb > 1
    torch.testing.assert_close(g0, g1)          # all-reduced grads agree
    torch.testing.assert_close(w0, w1)          # params identical after the step


def test_new_op_references_cpu():
    """CPU paths of the DLRM / detection / RoPE ops (the GPU kernels are pinned to these)."""
    from cloudtik_amd import ops
    from cloudtik_amd.ops.rope import rope_reference
    cos, sin = ops.rotary_cache(16, 8)
    x = torch.randn(2, 5, 3, 8, dtype=torch.bfloat16)
    q, k = ops.apply_rotary(x, x, cos, sin)
    back = rope_reference(q.reshape(-1, 3, 8).float(), cos, sin, torch.arange(10) % 5, inverse=True)
    assert torch.allclose(back, x.reshape(-1, 3, 8).float(), atol=0.05)
    ebc = ops.EmbeddingBagCollection([10, 20], 4)
    idx, offs = ops.pack_bags([torch.tensor([1, 2, 3]), torch.tensor([5])], [torch.tensor([0, 1]), torch.tensor([0, 0])], 2)
    out = ebc(idx, offs, 2)
    ref = torch.nn.functional.embedding_bag(torch.tensor([1, 2, 3]), ebc.weight[:10], torch.tensor([0, 1]), mode="sum")
    assert torch.allclose(out[:, 0], ref)
    assert torch.allclose(out[0, 1], torch.zeros(4)) and torch.allclose(out[1, 1], ebc.weight[15])
    z = ops.dot_interaction(torch.randn(3, 4), torch.randn(3, 2, 4))
    assert z.shape == (3, 4 + 3)
    boxes = torch.tensor([[0, 0, 10, 10], [1, 1, 11, 11], [50, 50, 60, 60.]])
    assert ops.nms(boxes, torch.tensor([0.5, 0.9, 0.1]), 0.5).tolist() == [1, 2]
    ra = ops.roi_align(torch.arange(16.).view(1, 1, 4, 4), torch.tensor([[0, 0, 0, 3, 3.]]), 1, aligned=False)
    assert abs(ra.item() - 7.5) < 1e-4   # mean of a linear ramp over the box
    fl = ops.sigmoid_focal_loss(torch.zeros(2, 3), torch.tensor([1, 0]))
    assert fl.item() > 0


def test_dropout_sites_with_close_keys_are_independent(monkeypatch):
    """Two dropout sites whose stream keys differ only in low bits must not draw permuted
    copies of one mask (mix32(ctr ^ key) would: site2[c] == site1[c ^ (k1 ^ k2)])."""
    import numpy as np
    n, p = 1 << 16, 0.5
    k1 = 0x12345670
    masks = []
    for k in (k1, k1 ^ 0x5):
        monkeypatch.setattr(R, "_dropout_key", lambda s, o, k=k: k)
        masks.append(R.dropout_keep_mask(n, p, seed=1, offset=0).numpy().reshape(-1, 2))
    m1, m2 = masks                                    # [pair counter, 2] 16-bit uniforms per hash
    ctr = np.arange(m1.shape[0])
    permuted = m1[(ctr ^ 0x5) % m1.shape[0]]
    assert (permuted == m2).mean() < 0.6              # independent: ~0.5 agreement per element
    assert abs((m1 == m2).mean() - 0.5) < 0.02


def test_wgrad_split_choice_fills_whole_waves():
    """tn2_splits (ops/linear.py): K loop (256-workgroup waves) + fp32 slab round trip --
    BERT-large qkv 48 tiles -> 5 (240 workgroups in one wave, a third of the slab bytes of 16),
    proj 16 -> 16, FFN 64 -> 4 -- and never fewer than 512 tokens per split."""
    import importlib
    L = importlib.import_module("cloudtik_amd.ops.linear")
    T = 32768
    assert L.tn2_splits(T, 3072, 1024) == 5
    assert L.tn2_splits(T, 1024, 1024) == 16
    assert L.tn2_splits(T, 4096, 1024) == 4 and L.tn2_splits(T, 1024, 4096) == 4
    assert L.tn2_splits(T, 8192, 8192) == 1                     # 1024 tiles: already 4 full waves
    assert L.tn2_splits(1024, 1024, 1024) == 2                   # >= 512 tokens per split
    assert L.tn2_splits(768, 1024, 1024) == 1
    for T_ in (4096, 32768, 65536):
        for N, K in ((1024, 1024), (3072, 1024), (4096, 1024), (768, 3072)):
            S = L.tn2_splits(T_, N, K)
            assert T_ // 64 >= S and (S == 1 or T_ // S >= 512)
