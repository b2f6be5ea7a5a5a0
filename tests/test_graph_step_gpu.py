"""Whole-step hipGraph capture (train/graph_step.py): a small ResNet trained through captured
replays follows the eager run step for step (weights, loss, BN running stats), with the
gradient side stream on; LAMB's per-step bias corrections reach the replays through the
optimizer's graph slot."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(seed=0):
    from cloudtik_amd.models.resnet import ResNetTrainStep, resnet18_like_small
    from cloudtik_amd.train.optim import FlatParamSpace, FusedSGD
    torch.manual_seed(seed)
    m = resnet18_like_small(device="cuda")
    m.train()
    named = list(m.named_parameters())
    sp = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
    opt = FusedSGD(sp, lr=0.05, momentum=0.9, weight_decay=1e-4, space=sp)
    g = torch.Generator().manual_seed(3)
    dt = next(m.parameters()).dtype
    x = torch.randn(8, 3, 32, 32, generator=g).to("cuda", dt).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), generator=g).cuda()
    return m, sp, opt, ResNetTrainStep(m, opt), x, y


def test_graphed_resnet_step_matches_eager():
    from cloudtik_amd.train.graph_step import GraphedStep
    m0, sp0, _, ts0, x, y = _setup()
    losses0 = [float(ts0(x, y).detach()) for _ in range(7)]
    m1, sp1, opt1, ts1, x1, y1 = _setup()
    step = GraphedStep(lambda: ts1(x1, y1), optimizers=[opt1], warmup=2)
    losses1 = [float(step().detach()) for _ in range(7)]
    assert step.graph is not None
    torch.testing.assert_close(torch.tensor(losses1), torch.tensor(losses0), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(sp1.model.float(), sp0.model.float(), rtol=5e-2, atol=5e-3)
    bn0 = [b for n, b in m0.named_buffers() if n.endswith("running_mean")]
    bn1 = [b for n, b in m1.named_buffers() if n.endswith("running_mean")]
    for a, b in zip(bn1, bn0):
        torch.testing.assert_close(a.float(), b.float(), rtol=5e-2, atol=5e-3)


def test_graph_slot_carries_per_step_bias_corrections():
    from cloudtik_amd.train.graph_step import GraphedStep
    from cloudtik_amd.train.optim import FlatParamSpace, FusedLAMB
    torch.manual_seed(1)
    w = torch.nn.Parameter(torch.randn(4096, device="cuda"))
    sp = FlatParamSpace([w], names=["w"])
    opt = FusedLAMB(sp, lr=1e-2, space=sp)
    target = torch.randn(4096, device="cuda")

    def body():
        loss = ((w - target) ** 2).sum()
        loss.backward()
        opt.step()
        opt.zero_grad()
        return loss

    w_ref = torch.nn.Parameter(w.detach().clone())
    sp_ref = FlatParamSpace([w_ref], names=["w"])
    opt_ref = FusedLAMB(sp_ref, lr=1e-2, space=sp_ref)
    for _ in range(8):
        ((w_ref - target) ** 2).sum().backward()
        opt_ref.step()
        opt_ref.zero_grad()
    step = GraphedStep(body, optimizers=[opt], warmup=2)
    for _ in range(8):
        step()
    torch.cuda.synchronize()
    assert opt.step_count == opt_ref.step_count == 8
    torch.testing.assert_close(w.detach(), w_ref.detach(), rtol=1e-5, atol=1e-6)
