"""DLRM hybrid parallelism on gloo: 2 ranks (tables sharded, all-to-all exchange, DP MLPs)
must produce the same loss and gradients as one process on the global batch."""
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


def _grads(model, world):
    dense = {n: p.grad.clone() for n, p in model.named_parameters() if not n.startswith("emb.")}
    return dense, model.emb.weight.grad.clone()


def _run(rank, world, port, out, B=16):
    import torch.distributed as dist
    from cloudtik_amd.models.dlrm import DLRM, DLRMConfig, synthetic_batch
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = DLRMConfig.tiny()
    torch.manual_seed(0)                               # identical dense init on every rank
    model = DLRM(cfg, rank=rank, world=world)
    dense, labels, idx, offs = synthetic_batch(cfg, B, step=3, tables=model.local_tables)
    Bl = B // world
    sl = slice(rank * Bl, (rank + 1) * Bl)
    logits = model(dense[sl], idx, offs, B)
    # global objective = mean over the global batch; each rank contributes its share
    loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, labels[sl]) / world
    loss.backward()
    dg, eg = _grads(model, world)
    if world > 1:
        for g in dg.values():
            dist.all_reduce(g)                         # DP part: sum of the per-rank shares
        t = torch.tensor([loss.item()])
        dist.all_reduce(t)
        lv = t.item()
    else:
        lv = loss.item()
    out[rank] = {"loss": lv, "dense": dg, "emb": eg, "tables": model.local_tables,
                 "logits": logits.detach(), "emb_weight": model.emb.weight.detach().clone()}
    if world > 1:
        dist.destroy_process_group()


def test_shard_tables_balanced():
    from cloudtik_amd.models.dlrm import shard_tables
    b = shard_tables([10, 10, 10, 10, 100, 10], 3)
    assert b[0][0] == 0 and b[-1][1] == 6 and all(hi > lo for lo, hi in b)
    assert all(b[i][1] == b[i + 1][0] for i in range(2))


def test_dlrm_hybrid_parallel_matches_single_process():
    single = {}
    _run(0, 1, 0, single)
    ctx = mp.get_context("spawn")
    with ctx.Manager() as m:
        out = m.dict()
        port = _port()
        ps = [ctx.Process(target=_run, args=(r, 2, port, out)) for r in range(2)]
        [p.start() for p in ps]
        [p.join(120) for p in ps]
        assert all(p.exitcode == 0 for p in ps)
        res = [dict(out[0]), dict(out[1])]
    ref = single[0]
    assert abs(res[0]["loss"] - ref["loss"]) < 1e-5
    torch.testing.assert_close(torch.cat([res[0]["logits"], res[1]["logits"]]), ref["logits"], atol=1e-5, rtol=1e-5)
    for k, g in ref["dense"].items():
        torch.testing.assert_close(res[0]["dense"][k], g, atol=1e-5, rtol=1e-4)
    # embedding grads: each rank owns a block of tables; together they equal the full grad
    from cloudtik_amd.models.dlrm import DLRMConfig
    sizes = DLRMConfig.tiny().table_sizes
    starts = [sum(sizes[:t]) for t in range(len(sizes))]
    full = ref["emb"]
    for r in res:
        rows = torch.cat([torch.arange(starts[t], starts[t] + sizes[t]) for t in r["tables"]])
        torch.testing.assert_close(r["emb"], full[rows], atol=1e-6, rtol=1e-4)
        torch.testing.assert_close(r["emb_weight"], ref["emb_weight"][rows])
