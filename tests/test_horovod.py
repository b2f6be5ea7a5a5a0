"""Horovod-compatible API on gloo (2 ranks): DistributedOptimizer == large-batch SGD,
compression, Adasum rule, collectives."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import cloudtik_amd.parallel.horovod as hvd
    hvd.init()
    res = {"rank": hvd.rank(), "size": hvd.size()}
    torch.manual_seed(rank)                      # different init -> broadcast_parameters must fix it
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 2))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(opt, root_rank=0)
    dopt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(),
                                    compression=hvd.Compression.none, fusion_threshold=256)
    g = torch.Generator().manual_seed(42)
    X, Y = torch.randn(8, 8, generator=g), torch.randn(8, 2, generator=g)
    x, y = X[rank * 4:(rank + 1) * 4], Y[rank * 4:(rank + 1) * 4]
    loss = torch.nn.functional.mse_loss(model(x), y)
    dopt.zero_grad()
    loss.backward()
    dopt.step()
    res["params"] = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    # collectives
    t = torch.tensor([float(rank + 1)])
    res["sum"] = hvd.allreduce(t, op=hvd.Sum).item()
    res["avg"] = hvd.allreduce(t).item()
    res["bf16"] = hvd.allreduce(torch.tensor([1.5]), compression=hvd.Compression.bf16, op=hvd.Sum).item()
    res["gather"] = hvd.allgather(torch.full((rank + 1, 2), float(rank))).tolist()
    res["bcast"] = hvd.broadcast_object({"r": rank}, root_rank=1)
    a = torch.tensor([1.0, 0.0]) if rank == 0 else torch.tensor([1.0, 1.0])
    res["adasum"] = hvd.allreduce(a, op=hvd.Adasum).tolist()
    out[rank] = res
    hvd.shutdown()


def test_horovod_api_two_ranks():
    ctx = mp.get_context("spawn")
    with ctx.Manager() as m:
        out = m.dict()
        port = _port()
        ps = [ctx.Process(target=_worker, args=(r, 2, port, out)) for r in range(2)]
        [p.start() for p in ps]
        [p.join(120) for p in ps]
        assert all(p.exitcode == 0 for p in ps)
        r0, r1 = dict(out[0]), dict(out[1])
    assert torch.allclose(r0["params"], r1["params"])
    # single-process reference on the full batch
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 2))
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(42)
    X, Y = torch.randn(8, 8, generator=g), torch.randn(8, 2, generator=g)
    torch.nn.functional.mse_loss(model(X), Y).backward()
    opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    assert torch.allclose(r0["params"], ref, atol=1e-6)
    assert r0["sum"] == 3.0 and r0["avg"] == 1.5 and r0["bf16"] == 3.0
    assert r0["gather"] == [[0.0, 0.0], [1.0, 1.0], [1.0, 1.0]]
    assert r0["bcast"] == {"r": 1}
    # Adasum of a=(1,0), b=(1,1): a.b=1, |a|^2=1, |b|^2=2 -> 0.5 a + 0.75 b = (1.25, 0.75)
    assert torch.allclose(torch.tensor(r0["adasum"]), torch.tensor([1.25, 0.75]))
    assert r0["adasum"] == r1["adasum"]
