"""RNN-T: transducer loss reference vs brute-force path enumeration, the
HIP lattice kernels vs the fp32 reference (loss and logits gradient), and the MLPerf-topology
model (train step, greedy decoding)."""
import itertools
import math

import pytest
import torch

from cloudtik_amd import ops
from cloudtik_amd.models.rnnt import RNNT, RNNTConfig, synthetic_speech_batch


def _brute_force_nll(logits, labels, T, U, blank):
    """Sum over every monotone lattice path: T blanks and U labels, ending with a blank."""
    lp = torch.log_softmax(logits.double(), -1)
    total = []
    # a path is the sequence of moves (b = blank: t+1, l = label: u+1); the last move is b
    for moves in set(itertools.permutations("b" * (T - 1) + "l" * U)):
        t = u = 0
        s = 0.0
        for mv in moves:
            if mv == "b":
                s += lp[t, u, blank]
                t += 1
            else:
                s += lp[t, u, labels[u]]
                u += 1
        s += lp[T - 1, U, blank]
        total.append(s)
    return -torch.logsumexp(torch.stack([torch.as_tensor(v) for v in total]), 0)


def test_reference_matches_path_enumeration():
    torch.manual_seed(0)
    for T, U in ((1, 0), (2, 1), (3, 2), (4, 3)):
        x = torch.randn(1, T, U + 1, 5)
        y = torch.randint(1, 5, (1, max(U, 1)))
        got = ops.rnnt_loss_reference(x, y, torch.tensor([T]), torch.tensor([U]), blank=0)
        want = _brute_force_nll(x[0], y[0].tolist(), T, U, 0)
        assert abs(float(got) - float(want)) < 1e-5, (T, U)


def test_reference_gradient_is_softmax_minus_occupancy():
    """Gradient rows sum to zero (softmax minus a distribution over transitions)."""
    torch.manual_seed(1)
    x = torch.randn(2, 4, 3, 6, requires_grad=True)
    y = torch.randint(0, 5, (2, 2))
    loss = ops.rnnt_loss_reference(x, y, torch.tensor([4, 3]), torch.tensor([2, 1]), blank=5).sum()
    loss.backward()
    assert torch.allclose(x.grad.sum(-1), torch.zeros(2, 4, 3), atol=1e-5)


def test_rnnt_model_train_and_decode_cpu():
    torch.manual_seed(0)
    cfg = RNNTConfig.tiny()
    m = RNNT(cfg, dtype=torch.float32)
    feats, flen, labels, llen = synthetic_speech_batch(3, T=16, U=4, cfg=cfg)
    opt = torch.optim.Adam(m.parameters(), lr=3e-3)
    first = None
    for _ in range(25):
        loss = m(feats, flen, labels, llen)
        first = float(loss) if first is None else first
        opt.zero_grad()
        loss.backward()
        opt.step()
    assert float(loss) < first * 0.8
    m.eval()
    hyps = m.greedy_decode(feats, flen)
    assert len(hyps) == 3 and all(all(0 <= k < cfg.vocab - 1 for k in h) for h in hyps)


def test_mlperf_rnnt_param_count():
    m = RNNT(RNNTConfig(), dtype=torch.float32)
    n = sum(p.numel() for p in m.parameters())
    assert 45e6 < n < 52e6          # MLPerf RNN-T is ~49M parameters


# --------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_rnnt_loss_hip_matches_reference(cuda, dtype):
    g = torch.Generator().manual_seed(3)
    B, T, U, V = 4, 23, 9, 37
    x = torch.randn(B, T, U + 1, V, generator=g).to(dtype)
    y = torch.randint(0, V - 1, (B, U), generator=g)
    tl = torch.tensor([23, 17, 1, 20])
    ul = torch.tensor([9, 4, 3, 0])
    xr = x.float().clone().requires_grad_()
    ref = ops.rnnt_loss_reference(xr, y, tl, ul, blank=V - 1)
    gw = torch.rand(B, generator=g) + 0.5
    (ref * gw).sum().backward()
    xg = x.to(cuda).requires_grad_()
    got = ops.rnnt_loss(xg, y.to(cuda), tl, ul, blank=V - 1, reduction="none")
    (got * gw.to(cuda)).sum().backward()
    torch.testing.assert_close(got.cpu(), ref.detach(), atol=1e-3, rtol=1e-4)
    tol = dict(atol=1e-5, rtol=1e-4) if dtype == torch.float32 else dict(atol=1e-2, rtol=2e-2)
    torch.testing.assert_close(xg.grad.float().cpu(), xr.grad.to(dtype).float(), **tol)


@pytest.mark.gpu
def test_rnnt_model_bf16_gpu(cuda):
    torch.manual_seed(0)
    cfg = RNNTConfig(enc_hidden=256, pred_hidden=128, joint_hidden=128)
    m = RNNT(cfg, device=cuda)
    feats, flen, labels, llen = synthetic_speech_batch(4, T=64, U=12, cfg=cfg, device=cuda)
    loss = m(feats, flen, labels, llen)
    loss.backward()
    assert torch.isfinite(loss) and torch.isfinite(m.joint_out.weight.grad.float()).all()
    m.eval()
    hyps = m.greedy_decode(feats, flen, max_symbols_per_step=3)
    assert len(hyps) == 4
