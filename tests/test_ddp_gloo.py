"""Data-parallel gradient reduction (parallel.GradBucketer) against single-process
full-batch gradients, over gloo with 2, 4 and 8 ranks (8 = one MI355X node): several buckets, an unused parameter,
``no_sync`` gradient accumulation over 2 micro-batches, bf16 gradients with fp32 reduction,
and the optimizer step that follows (reference semantics: DDP averaging,
ssd-resnet34 distributed.py:13-48, transfer-learning trainer.py:215-219)."""
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


class Net(torch.nn.Module):
    """``native``: the hidden layers go through ops.linear (weight gradient accumulated into the
    flat buffer on the gradient side stream, readiness reported via _ct_grad_ready) -- the
    path BERT's layers take on the GPU."""

    def __init__(self, native=False):
        super().__init__()
        self.native = native
        self.fc1 = torch.nn.Linear(16, 32)
        self.fc2 = torch.nn.Linear(32, 32)
        self.unused = torch.nn.Linear(8, 8)     # never receives a gradient
        self.head = torch.nn.Linear(32, 4)

    def forward(self, x):
        if self.native:
            from cloudtik_amd.ops.linear import linear
            h = torch.relu(linear(x, self.fc1.weight, self.fc1.bias))
            return self.head(torch.relu(linear(h, self.fc2.weight, self.fc2.bias)))
        return self.head(torch.relu(self.fc2(torch.relu(self.fc1(x)))))


GLOBAL_B = 32


def _data():
    g = torch.Generator().manual_seed(5)
    return torch.randn(GLOBAL_B, 16, generator=g), torch.randint(0, 4, (GLOBAL_B,), generator=g)


def _make(dtype, device="cpu"):
    torch.manual_seed(0)
    return Net(native=device == "cuda").to(dtype).to(device)


def _worker(rank, world, port, accum, fp32_reduce, out, device="cpu"):
    import torch.distributed as dist
    from contextlib import nullcontext
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FlatParamSpace, FusedSGD
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if device == "cuda":
        torch.cuda.set_device(0)             # every rank shares GPU 0; gloo moves the tensors
    try:
        dtype = torch.bfloat16 if fp32_reduce else torch.float32
        model = _make(dtype, device)
        if rank:                                 # rank-local init differs: the broadcast must fix it
            with torch.no_grad():
                for p in model.parameters():
                    p.add_(1.0)
        named = list(model.named_parameters())
        space = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
        opt = FusedSGD(space, lr=0.1, momentum=0.0, space=space)
        broadcast_flat_params(space)
        ddp = GradBucketer(space, bucket_mb=0.0004, reduce_dtype=torch.float32 if fp32_reduce else None)
        opt.grad_scale = ddp.grad_scale / accum
        X, Y = _data()
        n = GLOBAL_B // world
        xs, ys = X[rank * n:(rank + 1) * n].to(dtype).to(device), Y[rank * n:(rank + 1) * n].to(device)
        m = n // accum
        for i in range(accum):
            ctx = ddp.no_sync() if i < accum - 1 else nullcontext()
            with ctx:
                loss = torch.nn.functional.cross_entropy(model(xs[i * m:(i + 1) * m]).float(), ys[i * m:(i + 1) * m])
                loss.backward()
        ddp.finish()
        g = space.reduced_grad.float() * opt.grad_scale
        grads = {nm: g[o:o + k].cpu().clone() for nm, o, k in zip(space.names, space.offsets, space.numels)}
        opt.step()
        params = {nm: p.detach().float().reshape(-1).cpu().clone() for nm, p in named}
        out[rank] = (grads, params, len(ddp.buckets))
    finally:
        dist.destroy_process_group()


def _reference():
    model = _make(torch.float32)
    X, Y = _data()
    torch.nn.functional.cross_entropy(model(X), Y).backward()
    grads = {n: (p.grad.reshape(-1).clone() if p.grad is not None else torch.zeros(p.numel()))
             for n, p in model.named_parameters()}
    params = {n: (p.detach() - 0.1 * p.grad).reshape(-1) if p.grad is not None else p.detach().reshape(-1)
              for n, p in model.named_parameters()}
    return grads, params


@pytest.mark.parametrize("world,accum,fp32_reduce", [(2, 1, False), (2, 2, False), (4, 2, False), (2, 2, True),
                                                     (4, 1, True), (8, 1, False), (8, 2, True)])
def test_gradbucketer_matches_full_batch(world, accum, fp32_reduce, device="cpu"):
    port = _port()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        procs = [ctx.Process(target=_worker, args=(r, world, port, accum, fp32_reduce, out, device))
                 for r in range(world)]
        [p.start() for p in procs]
        [p.join(180) for p in procs]
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res = dict(out)
    ref_g, ref_p = _reference()
    tol = dict(rtol=3e-2, atol=3e-3) if fp32_reduce else (dict(rtol=1e-5, atol=1e-6) if device == "cpu"
                                                          else dict(rtol=1e-4, atol=1e-5))
    for r in range(world):
        grads, params, nb = res[r]
        assert nb > 2
        for n in ref_g:
            torch.testing.assert_close(grads[n], ref_g[n], **tol, msg=f"rank {r} grad {n}")
            torch.testing.assert_close(params[n], ref_p[n], **tol, msg=f"rank {r} param {n}")
        assert torch.count_nonzero(grads["unused.weight"]) == 0
    for n in ref_g:                              # bit-identical across ranks
        assert torch.equal(res[0][1][n], res[world - 1][1][n])


@pytest.mark.gpu
@pytest.mark.parametrize("accum,fp32_reduce", [(1, False), (2, False), (2, True)])
def test_gradbucketer_matches_full_batch_gpu(accum, fp32_reduce):
    """The GPU data-parallel path: two ranks on GPU 0, ops.linear weight gradients from the
    side stream into the flat buffer, bucket launches from the readiness callbacks."""
    test_gradbucketer_matches_full_batch(2, accum, fp32_reduce, device="cuda")
