"""Multi-GPU readiness checks that run on the CPU (gloo), for the data-parallel paths the 8-GPU
bench takes (parallel/ddp.py GradBucketer, train/optim.py FlatParamSpace + fused optimizers):

* overlap ordering: with world > 1 the first gradient bucket's collective is issued from the
  gradient hooks while backward is still producing earlier layers' gradients -- not after it;
* 4-rank ZeRO-1 (reduce-scatter + sharded optimizer + all-gather) with fp32 gradient
  reduction for the tiny BERT (LAMB) and tiny ResNet (SGD) of bench.py --model tiny equals the
  single-process update on the same per-rank micro-batches with averaged gradients (the data-
  parallel semantics: per-rank BatchNorm statistics, mean gradient)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _overlap_worker(rank, world, port, out):
    import torch.distributed as dist
    from cloudtik_amd.parallel import GradBucketer
    from cloudtik_amd.train.optim import FlatParamSpace
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        layers = [torch.nn.Linear(64, 64) for _ in range(6)]
        model = torch.nn.Sequential(*[m for l in layers for m in (l, torch.nn.Tanh())])
        named = list(model.named_parameters())
        space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
        ddp = GradBucketer(space, bucket_mb=64 * 65 * 4 / 2 ** 20)       # about one layer per bucket
        events = []
        orig = ddp._launch

        def launch(b):
            events.append(("bucket", b))
            return orig(b)

        ddp._launch = launch
        # the first layer's weight gradient is the last one backward produces
        layers[0].weight.register_post_accumulate_grad_hook(lambda p: events.append(("first_layer_grad", 0)))
        x = torch.randn(8, 64)
        model(x).square().mean().backward()
        ddp.finish()
        out[rank] = (events, len(ddp.buckets))
    finally:
        dist.destroy_process_group()


def test_first_bucket_launches_before_backward_ends():
    port = _port()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        ps = [ctx.Process(target=_overlap_worker, args=(r, 2, port, out)) for r in range(2)]
        [p.start() for p in ps]
        [p.join(120) for p in ps]
        assert all(p.exitcode == 0 for p in ps)
        res = dict(out)
    for r in range(2):
        events, nb = res[r]
        assert nb >= 4
        kinds = [k for k, _ in events]
        last_grad = kinds.index("first_layer_grad")
        launched_before = [e for e in events[:last_grad] if e[0] == "bucket"]
        # buckets are issued in order, most of them while backward is still running
        assert launched_before and launched_before[0] == ("bucket", 0)
        assert len(launched_before) >= nb - 2
        assert [b for k, b in events if k == "bucket"] == list(range(nb))


def _batches(kind, world, step, B=8):
    from cloudtik_amd.models.bert import BertConfig, synthetic_pretraining_batch
    out = []
    for r in range(world):
        g = torch.Generator().manual_seed(100 * step + r)
        if kind == "bert":
            out.append(synthetic_pretraining_batch(BertConfig.tiny(), 2, 32, 5, device="cpu", generator=g))
        else:
            out.append((torch.randn(B, 3, 64, 64, generator=g), torch.randint(0, 10, (B,), generator=g)))
    return out


def _build(kind, dtype=torch.float32):
    torch.manual_seed(1234)
    if kind == "bert":
        from cloudtik_amd.models.bert import BertConfig, BertForPreTraining
        cfg = BertConfig.tiny(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        m = BertForPreTraining(cfg, dtype=dtype)
    else:
        from cloudtik_amd.models.resnet import resnet18_like_small
        m = resnet18_like_small().to(dtype)
    m.train()
    return m


def _loss(kind, model, batch):
    if kind == "bert":
        return model(**batch)
    x, y = batch
    return torch.nn.functional.cross_entropy(model(x.to(next(model.parameters()).dtype)).float(), y)


def _optimizer(kind, space):
    from cloudtik_amd.train.optim import FusedLAMB, FusedSGD
    if kind == "bert":
        return FusedLAMB(space, lr=1e-2, weight_decay=0.01, no_decay=lambda n: n.endswith("bias"), space=space)
    return FusedSGD(space, lr=0.05, momentum=0.9, weight_decay=1e-4, space=space)


def _zero_worker(rank, world, port, kind, dtype, out):
    import torch.distributed as dist
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FlatParamSpace
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _build(kind, dtype)
        named = list(model.named_parameters())
        space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named], shard=(rank, world))
        opt = _optimizer(kind, space)
        broadcast_flat_params(space)
        ddp = GradBucketer(space, bucket_mb=0.05, reduce_dtype=torch.float32, mode="reduce_scatter")
        opt.grad_scale = ddp.grad_scale
        assert space.sharded and len(ddp.buckets) > 2
        for step in range(2):
            _loss(kind, model, _batches(kind, world, step)[rank]).backward()
            ddp.finish()
            opt.step()
            opt.zero_grad()
        out[rank] = {n: p.detach().clone() for n, p in named}
    finally:
        dist.destroy_process_group()


def _single_process_reference(kind, world, dtype):
    """Same updates in one process: per-rank micro-batch gradients averaged, one optimizer
    step per step."""
    from cloudtik_amd.train.optim import FlatParamSpace
    model = _build(kind, dtype)
    named = list(model.named_parameters())
    space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = _optimizer(kind, space)
    for step in range(2):
        acc = torch.zeros_like(space.grad, dtype=torch.float32)
        for b in _batches(kind, world, step):
            space.grad.zero_()
            _loss(kind, model, b).backward()
            acc += space.grad.float()
        space.grad.copy_(acc / world)
        opt.step()
        opt.zero_grad()
    return {n: p.detach().clone() for n, p in named}


@pytest.mark.parametrize("kind,dtype", [("bert", torch.float32), ("resnet", torch.float32),
                                        ("bert", torch.bfloat16), ("resnet", torch.bfloat16)])
def test_zero1_fp32_reduce_four_ranks_matches_single_process(kind, dtype):
    """fp32 models: exact data-parallel semantics.  bf16 models (the bench's configuration:
    bf16 weights, fp32 master shard, fp32 gradient reduction): the ranks reduce unrounded fp32
    sums while the reference rounds the averaged gradient to bf16, so the weights may differ by
    about one bf16 ulp."""
    world = 4
    port = _port()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        ps = [ctx.Process(target=_zero_worker, args=(r, world, port, kind, dtype, out)) for r in range(world)]
        [p.start() for p in ps]
        [p.join(300) for p in ps]
        assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
        res = dict(out)
    ref = _single_process_reference(kind, world, dtype)
    for r in range(world):
        for n, v in ref.items():
            assert res[r][n].dtype == dtype
            if dtype == torch.float32:
                torch.testing.assert_close(res[r][n], v, rtol=2e-4, atol=2e-5, msg=f"rank {r} {n}")
        if dtype != torch.float32:
            # bf16 weights: within one bf16 ulp almost everywhere (an Adam-type step on a
            # near-zero gradient may flip sign under rounding; updates far below one ulp of the
            # weight are quantisation, hence no whole-update norm comparison)
            a = torch.cat([res[r][n].float().reshape(-1) for n in ref])
            b = torch.cat([ref[n].float().reshape(-1) for n in ref])
            off = (a - b).abs() > 8e-3 * b.abs() + 1e-5
            assert off.float().mean().item() < 1e-2, off.float().mean().item()
        for n in ref:                                 # every rank holds the same (all-gathered) weights
            assert torch.equal(res[r][n], res[0][n])
