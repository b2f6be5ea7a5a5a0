"""ZeRO-1 (GradBucketer(mode="reduce_scatter") + FlatParamSpace(shard=(rank, world))) is
the same optimizer as the unsharded all-reduce path: identical weights after several steps
(LAMB with its cross-shard per-tensor trust-ratio norms, AdamW, SGD), optimizer state saved in
the global layout (equal to the unsharded run's state), and resume from such a checkpoint
continues bit-for-bit.  gloo, 2 and 4 ranks."""
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


def _model(dtype):
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(20, 48), torch.nn.GELU(), torch.nn.LayerNorm(48),
                               torch.nn.Linear(48, 40), torch.nn.GELU(), torch.nn.Linear(40, 5)).to(dtype)


def _build(kind, dtype, rank, world, zero):
    from cloudtik_amd.parallel import GradBucketer, broadcast_flat_params
    from cloudtik_amd.train.optim import FlatParamSpace, FusedAdam, FusedLAMB, FusedSGD
    m = _model(dtype)
    named = list(m.named_parameters())
    sp = FlatParamSpace([p for _, p in named], names=[n for n, _ in named],
                        shard=(rank, world) if zero else (0, 1))
    nd = lambda n: n.endswith("bias") or n.startswith("2.")  # noqa: E731
    if kind == "lamb":
        opt = FusedLAMB(sp, lr=1e-2, weight_decay=0.01, no_decay=nd, space=sp)
    elif kind == "adamw":
        opt = FusedAdam(sp, lr=1e-2, weight_decay=0.01, no_decay=nd, space=sp)
    else:
        opt = FusedSGD(sp, lr=0.05, momentum=0.9, weight_decay=1e-4, space=sp)
    broadcast_flat_params(sp)
    ddp = GradBucketer(sp, bucket_mb=0.0006, mode="reduce_scatter" if zero else "all_reduce")
    opt.grad_scale = ddp.grad_scale
    return m, sp, opt, ddp


def _steps(m, opt, ddp, rank, dtype, its):
    for it in its:
        g = torch.Generator().manual_seed(1000 * it + rank)
        x = torch.randn(12, 20, generator=g).to(dtype)
        m(x).float().pow(2).mean().backward()
        ddp.finish()
        opt.step()
        opt.zero_grad()


def _real(sp, t):
    """Only the parameter elements of a global-layout flat tensor (padding differs by world)."""
    return torch.cat([t[o:o + n] for o, n in zip(sp.offsets, sp.numels)]).float().clone()


def _worker(rank, world, port, kind, dtype, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        m0, sp0, opt0, ddp0 = _build(kind, dtype, rank, world, zero=False)
        _steps(m0, opt0, ddp0, rank, dtype, range(3))
        res["plain"] = _real(sp0, sp0.model)
        res["plain_state"] = {k: _real(sp0, v) for k, v in opt0.state_dict()["flat"].items()}
        m1, sp1, opt1, ddp1 = _build(kind, dtype, rank, world, zero=True)
        assert sp1.sharded and len(ddp1.buckets) > 2
        _steps(m1, opt1, ddp1, rank, dtype, range(3))
        res["zero"] = _real(sp1, sp1.model)
        sd = opt1.state_dict()
        res["zero_state"] = {k: _real(sp1, v) for k, v in sd["flat"].items()}
        # resume: 2 steps, checkpoint (model + global-layout optimizer state), fresh run, 1 step
        m2, sp2, opt2, ddp2 = _build(kind, dtype, rank, world, zero=True)
        _steps(m2, opt2, ddp2, rank, dtype, range(2))
        ck = (sp2.model.clone(), opt2.state_dict())
        m3, sp3, opt3, ddp3 = _build(kind, dtype, rank, world, zero=True)
        sp3.model.copy_(ck[0])                 # what Checkpointer.load's model.load_state_dict does
        opt3.load_state_dict(ck[1])            # must refresh local_model / master itself
        _steps(m3, opt3, ddp3, rank, dtype, range(2, 3))
        res["resumed"] = _real(sp3, sp3.model)
        if rank == 0:                          # for the world-size-change check in the parent
            res["ckpt_model"] = ck[0].clone()
            res["ckpt_state"] = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in ck[1].items()
                                 if k in ("flat", "flat_layout", "flat_params", "step_count")}
            res["ckpt_state"]["full"] = opt2.state_dict()
        else:
            opt2.state_dict()                  # collective: every rank takes part
        out[rank] = res
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,world,dtype", [("lamb", 2, torch.float32), ("adamw", 4, torch.float32),
                                              ("sgd", 2, torch.float32), ("lamb", 4, torch.bfloat16),
                                              ("lamb", 8, torch.float32)])
def test_zero1_matches_unsharded(kind, world, dtype):
    port = _port()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        procs = [ctx.Process(target=_worker, args=(r, world, port, kind, dtype, out)) for r in range(world)]
        [p.start() for p in procs]
        [p.join(180) for p in procs]
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res = dict(out)
    tol = dict(rtol=1e-5, atol=1e-6) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-3)
    for r in range(world):
        torch.testing.assert_close(res[r]["zero"], res[r]["plain"], **tol)
        torch.testing.assert_close(res[r]["resumed"], res[r]["zero"], rtol=0, atol=0)
        for k, v in res[r]["plain_state"].items():
            torch.testing.assert_close(res[r]["zero_state"][k], v, **tol, msg=k)
    assert torch.equal(res[0]["zero"], res[world - 1]["zero"])
    # the global-layout state restores unsharded at world size 1 (other tail padding)
    from cloudtik_amd.train.optim import FlatParamSpace
    m1, sp1, opt1, _ = _build(kind, dtype, 0, 1, zero=False)
    assert sp1.total != res[0]["ckpt_model"].numel() or world == 1 or sp1.total % world == 0
    n = min(sp1.total, res[0]["ckpt_model"].numel())
    sp1.model[:n].copy_(res[0]["ckpt_model"][:n])
    opt1.load_state_dict(res[0]["ckpt_state"]["full"])
    saved = res[0]["ckpt_state"]["flat"]
    for k, v in opt1.state_dict()["flat"].items():
        torch.testing.assert_close(_real(sp1, v), _real(sp1, saved[k][:sp1.used].float()
                                   if saved[k].numel() >= sp1.used else saved[k]), rtol=0, atol=0, msg=k)
    assert isinstance(sp1, FlatParamSpace)


def _trainer_worker(rank, world, port, ckdir, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from cloudtik_amd.train.trainer import Trainer
    g = torch.Generator().manual_seed(5 + rank)
    x = torch.randn(96, 20, generator=g)
    y = torch.randint(0, 5, (96,), generator=g)
    batches = [(x[i:i + 16], y[i:i + 16]) for i in range(0, 96, 16)]
    try:
        def run(epochs, ck, seed):
            torch.manual_seed(seed)
            m = torch.nn.Sequential(torch.nn.Linear(20, 48), torch.nn.GELU(), torch.nn.Linear(48, 5))
            t = Trainer(m, "adamw", lr=1e-2, weight_decay=0.01, train_loader=batches, epochs=epochs, log_every=0,
                        checkpoint_dir=ck, zero=True, bucket_mb=0.002)
            assert t.space.sharded and t.space.master is None        # fp32: no master copy
            t.fit()
            return {k: v.detach().clone() for k, v in t.model.state_dict().items()}
        straight = run(2, None, 0)
        run(1, ckdir, 0)                       # checkpoint at the end of epoch 0
        resumed = run(2, ckdir, 123)           # other init: the checkpoint must overwrite it
        out[rank] = {"straight": straight, "resumed": resumed}
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_trainer_zero1_resume_fp32(tmp_path):
    """Trainer(zero=True) with fp32 parameters (no master copy) resumes from its checkpoint
    and ends on the same weights as an uninterrupted run."""
    port = _port()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as mgr:
        out = mgr.dict()
        procs = [ctx.Process(target=_trainer_worker, args=(r, 2, port, str(tmp_path), out)) for r in range(2)]
        [p.start() for p in procs]
        [p.join(240) for p in procs]
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res = dict(out)
    assert os.path.exists(os.path.join(str(tmp_path), "step-6", "optim.pt"))
    for r in range(2):
        for k, v in res[r]["straight"].items():
            torch.testing.assert_close(res[r]["resumed"][k], v, rtol=1e-6, atol=1e-7, msg=k)
