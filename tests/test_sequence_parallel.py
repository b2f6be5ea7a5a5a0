"""Sequence parallelism: ring attention and Ulysses over a gloo group of
2 and 4 CPU ranks must reproduce full attention (output and q/k/v gradients), causal and
not; the single-GPU block primitives must match the fp32 reference on the MI355X."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _full(q, k, v, causal):
    from cloudtik_amd.ops import reference as ref
    o = ref.attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), scale=1.0 / math.sqrt(q.shape[-1]),
                      causal=causal)
    return o.transpose(1, 2)


def _worker(rank, world, port, kind, causal, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from cloudtik_amd.parallel.sequence import ring_attention, ulysses_attention
    g = torch.Generator().manual_seed(0)
    B, S, H, D = 2, 8 * world, 4, 16
    q, k, v = (torch.randn(B, S, H, D, generator=g, dtype=torch.float64) for _ in range(3))
    go = torch.randn(B, S, H, D, generator=g, dtype=torch.float64)
    s = S // world
    sl = slice(rank * s, (rank + 1) * s)
    ql, kl, vl = (t[:, sl].clone().requires_grad_() for t in (q, k, v))
    fn = ring_attention if kind == "ring" else ulysses_attention
    o = fn(ql, kl, vl, causal=causal)
    (o * go[:, sl]).sum().backward()
    torch.save({"o": o.detach(), "dq": ql.grad, "dk": kl.grad, "dv": vl.grad},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["ring", "ulysses"])
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("causal", [False, True])
def test_sequence_parallel_matches_full_attention(tmp_path, kind, world, causal):
    mp.spawn(_worker, args=(world, _port(), kind, causal, str(tmp_path)), nprocs=world, join=True)
    g = torch.Generator().manual_seed(0)
    B, S, H, D = 2, 8 * world, 4, 16
    q, k, v = (torch.randn(B, S, H, D, generator=g, dtype=torch.float64).requires_grad_() for _ in range(3))
    go = torch.randn(B, S, H, D, generator=g, dtype=torch.float64)
    ref = _full(q, k, v, causal)
    (ref * go).sum().backward()
    parts = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    cat = {n: torch.cat([p[n] for p in parts], 1) for n in ("o", "dq", "dk", "dv")}
    tol = dict(atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(cat["o"].double(), ref.detach(), **tol)
    torch.testing.assert_close(cat["dq"].double(), q.grad, **tol)
    torch.testing.assert_close(cat["dk"].double(), k.grad, **tol)
    torch.testing.assert_close(cat["dv"].double(), v.grad, **tol)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_ring_block_kernels_gpu(cuda, causal):
    """The HIP block forward (LSE in natural log) and block backward with an external LSE
    match the fp32 block implementation."""
    from cloudtik_amd.parallel import sequence as SP
    g = torch.Generator().manual_seed(1)
    B, S, H, D = 2, 256, 4, 64
    q, k, v, do = (torch.randn(B, S, H, D, generator=g).to(cuda, torch.bfloat16) for _ in range(4))
    o, lse = SP.block_forward(q, k, v, 0.125, causal)
    qf, kf, vf = q.float(), k.float(), v.float()
    s = torch.einsum("bqhd,bkhd->bhqk", qf, kf) * 0.125
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=cuda).triu(1), float("-inf"))
    lse_ref = torch.logsumexp(s, -1)
    o_ref = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), vf)
    torch.testing.assert_close(lse, lse_ref, atol=2e-2, rtol=1e-3)
    torch.testing.assert_close(o, o_ref, atol=3e-2, rtol=3e-2)
    dq, dk, dv = SP.block_backward(q, k, v, o_ref.to(torch.bfloat16), do, lse_ref, 0.125, causal)
    p = torch.exp(s - lse_ref[..., None])
    dv_ref = torch.einsum("bhqk,bqhd->bkhd", p, do.float())
    torch.testing.assert_close(dv, dv_ref, atol=5e-2, rtol=5e-2)
    assert torch.isfinite(dq).all() and torch.isfinite(dk).all()
