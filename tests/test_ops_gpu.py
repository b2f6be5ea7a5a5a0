"""Numerics of every HIP kernel vs a plain-PyTorch fp32 reference of the same op (GPU)."""
import math

import pytest
import torch

from cloudtik_amd import ops
from cloudtik_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("N", [64, 768, 1024, 2048])
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("M", [333, 6151])
def test_layernorm_fwd_bwd(cuda, N, fused, M):
    """M 6151: more rows than the backward grid has waves (768 x 4 at N <= 1024), so every wave
    walks 2-3 rows through the prefetch pipeline, ending on either register set."""
    torch.manual_seed(0)
    x = torch.randn(M, N, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    res = torch.randn(M, N, device=cuda, dtype=torch.bfloat16, requires_grad=True) if fused else None
    bias = (torch.randn(N, device=cuda) * 0.1).bfloat16().requires_grad_(fused) if fused else None
    g = (1 + 0.1 * torch.randn(N, device=cuda)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(N, device=cuda)).bfloat16().requires_grad_()
    p = 0.1 if fused else 0.0
    ops.manual_seed(7)
    y = ops.layer_norm(x, g, b, 1e-12, bias=bias, residual=res, p=p, training=True)
    dy = torch.randn_like(y)
    y.backward(dy)
    grads = [t.grad.clone() for t in (x, g, b) + ((res, bias) if fused else ())]
    # reference with identical dropout stream
    xs = [t.detach().float().requires_grad_() for t in (x, g, b) + ((res, bias) if fused else ())]
    ops.manual_seed(7)
    seed, off = ops._rng.next(x.numel()) if p > 0 else (0, 0)
    yr, _ = ref.layer_norm(xs[0], xs[1], xs[2], 1e-12, xs[4] if fused else None,
                           xs[3] if fused else None, p, seed, off)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    for gk, xr in zip(grads, xs):
        assert _rel(gk, xr.grad) < 2e-2


@pytest.mark.parametrize("N", [768, 1024])
def test_layernorm_bwd_from_output(cuda, N):
    """The output-based LayerNorm backward (xhat = (y - beta) / gamma, csrc/layernorm.hip FROMY;
    what the BERT blocks run) against the fp32 reference, with gamma spread over [0.3, 1.7], beta
    over [-1, 1], and one gamma exactly 0 (that channel: xhat 0, so its dgamma is 0)."""
    C = ops.require_native()
    torch.manual_seed(1)
    M, p, eps = 333, 0.1, 1e-12
    x = torch.randn(M, N, device=cuda).bfloat16()
    res = torch.randn(M, N, device=cuda).bfloat16()
    bias = (0.1 * torch.randn(N, device=cuda)).bfloat16()
    g = (0.3 + 1.4 * torch.rand(N, device=cuda)).bfloat16()
    g[5] = 0
    b = (2 * torch.rand(N, device=cuda) - 1).bfloat16()
    dy = torch.randn(M, N, device=cuda).bfloat16()
    seed, off = 11, 4096
    y, s, mean, rstd = C.layernorm_fwd(x, bias, res, g, b, eps, False, p, seed, off, keep_sum=False)
    assert not s.defined() if hasattr(s, "defined") else s is None
    outs = {}
    for form in ("sum", "y"):
        y2, s2, mean2, rstd2 = C.layernorm_fwd(x, bias, res, g, b, eps, False, p, seed, off, keep_sum=form == "sum")
        assert torch.equal(y2, y)
        dg, db, dbias = (torch.zeros(N, device=cuda) for _ in range(3))
        ds, dx = C.layernorm_bwd_into(dy, y2 if form == "y" else s2, g, mean2, rstd2, False, dg, db, dbias, True,
                                      p, seed, off, beta_y=b if form == "y" else None)
        torch.cuda.synchronize()
        outs[form] = (ds, dx, dg, db, dbias)
    xs = [t.float().requires_grad_() for t in (x, g, b, res, bias)]
    yr, _ = ref.layer_norm(xs[0], xs[1], xs[2], eps, xs[4], xs[3], p, seed, off)
    yr.backward(dy.float())
    keep = torch.ones(N, dtype=torch.bool, device=cuda)
    keep[5] = False
    ds, dx, dg, db, dbias = outs["y"]
    assert torch.isfinite(ds.float()).all() and torch.isfinite(dx.float()).all()
    assert _rel(ds, xs[3].grad) < 2e-2 and _rel(dx, xs[0].grad) < 2e-2
    assert _rel(dg[keep], xs[1].grad[keep]) < 2e-2 and dg[5].item() == 0.0
    assert _rel(db, xs[2].grad) < 2e-2 and _rel(dbias, xs[4].grad) < 2e-2
    # and next to the saved-sum form, which the output form replaces
    for a_, b_ in zip(outs["y"][:2], outs["sum"][:2]):
        assert _rel(a_, b_) < 1e-2


@pytest.mark.parametrize("act", [ops.ACT_GELU, ops.ACT_RELU])
def test_bias_act(cuda, act):
    torch.manual_seed(0)
    z = torch.randn(257, 4096, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    bias = (0.1 * torch.randn(4096, device=cuda)).bfloat16().requires_grad_()
    y = ops.bias_act(z, bias, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    zr, br = z.detach().float().requires_grad_(), bias.detach().float().requires_grad_()
    yr = ref.bias_act(zr, br, act)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(z.grad, zr.grad) < 1e-2
    assert _rel(bias.grad, br.grad) < 1e-2


def test_dropout_matches_reference_mask(cuda):
    x = torch.randn(64, 1024, device=cuda, dtype=torch.bfloat16)
    ops.manual_seed(3)
    y = ops.dropout(x, 0.1, True)
    ops.manual_seed(3)
    seed, off = ops._rng.next(x.numel())
    yr = ref.dropout(x.float(), 0.1, seed, off)
    assert torch.equal((y == 0), (yr == 0))
    frac = (y == 0).float().mean().item()
    assert abs(frac - 0.1) < 0.01


@pytest.mark.parametrize("T,B,S,H", [(2, 4, 64, 256), (3, 16, 32, 320), (1, 64, 16, 1024)])
def test_embedding3(cuda, T, B, S, H):
    """Word / position / token-type gradients (per-position kernel: register sums for <= 2
    token types, atomics for more; columns not a multiple of the 256-column block)."""
    torch.manual_seed(0)
    V, P = 1000, 128
    W = torch.randn(V, H, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    Pe = torch.randn(P, H, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    Te = torch.randn(T, H, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    ids = torch.randint(0, V, (B, S), device=cuda)
    ids[:, 0] = 7                       # one id at a position in every sequence ([CLS])
    ids[: B // 2, -2:] = 0              # runs of one id down the batch (padding)
    tt = torch.randint(0, T, (B, S), device=cuda)
    y = ops.embedding3(ids, tt, W, Pe, Te)
    dy = torch.randn_like(y)
    y.backward(dy)
    Wr, Pr, Tr = (t.detach().float().requires_grad_() for t in (W, Pe, Te))
    yr = ref.embedding3(ids, tt, Wr, Pr, Tr)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    for a, b in ((W, Wr), (Pe, Pr), (Te, Tr)):
        assert _rel(a.grad, b.grad) < 2e-2


@pytest.mark.parametrize("R", [300, 320])     # 320 rows: decoder weight gradient on the MFMA TN kernel
def test_linear_cross_entropy(cuda, R):
    torch.manual_seed(0)
    H, V, Vp = 256, 1000, 1024
    x = torch.randn(R, H, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    W = (0.05 * torch.randn(Vp, H, device=cuda)).bfloat16().requires_grad_()
    b = (0.05 * torch.randn(Vp, device=cuda)).bfloat16().requires_grad_()
    labels = torch.randint(0, V, (R,), device=cuda)
    labels[::7] = -100
    loss = ops.cross_entropy_fused(x, W, b, labels, V=V)
    loss.backward()
    xr, Wr, br = (t.detach().float().requires_grad_() for t in (x, W, b))
    lr_ = torch.nn.functional.cross_entropy((xr @ Wr.t() + br)[:, :V], labels, ignore_index=-100)
    lr_.backward()
    assert abs(loss.item() - lr_.item()) < 2e-2 * abs(lr_.item())
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(W.grad[:V], Wr.grad[:V]) < 3e-2
    assert W.grad[V:].abs().max().item() == 0.0
    assert _rel(b.grad[:V], br.grad[:V]) < 3e-2           # 320 rows: from the TN kernel's all-ones MFMA
    assert b.grad[V:].abs().max().item() == 0.0


@pytest.mark.parametrize("S", [128, 64, 200, 512])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_packed(cuda, S, p):
    torch.manual_seed(0)
    B, H, D = 2, 4, 64
    qkv = (torch.randn(B, S, 3 * H * D, device=cuda) * 0.5).bfloat16().requires_grad_()
    mask = torch.ones(B, S, device=cuda)
    mask[1, S - S // 4:] = 0
    kb = (1.0 - mask) * -10000.0
    ops.manual_seed(11)
    o = ops.attention_packed(qkv, H, kb, p=p, training=True)
    do = torch.randn_like(o)
    o.backward(do)
    qr = qkv.detach().float().requires_grad_()
    v5 = qr.view(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
    ops.manual_seed(11)
    seed, off = ops._rng.next(B * H * S * S) if p > 0 else (0, 0)
    orf = ref.attention(v5[0], v5[1], v5[2], kb, p, seed, off).permute(0, 2, 1, 3).reshape(B, S, H * D)
    orf.backward(do.float())
    assert _rel(o, orf) < 2e-2
    assert _rel(qkv.grad, qr.grad) < 3e-2


def test_attention_bhsd_causal(cuda):
    torch.manual_seed(1)
    B, H, S, D = 2, 3, 96, 64
    q, k, v = (torch.randn(B, H, S, D, device=cuda).bfloat16().requires_grad_() for _ in range(3))
    o = ops.attention(q, k, v, causal=True)
    do = torch.randn_like(o)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = ref.attention(qr, kr, vr, causal=True)
    orf.backward(do.float())
    assert _rel(o, orf) < 2e-2
    for a, b in ((q, qr), (k, kr), (v, vr)):
        assert _rel(a.grad, b.grad) < 3e-2


@pytest.mark.parametrize("name", ["lamb", "adamw", "sgd"])
def test_fused_optimizers_match_torch_path(cuda, name):
    from cloudtik_amd.train.optim import FlatParamSpace, FusedLAMB, FusedAdam, FusedSGD
    torch.manual_seed(0)

    def make(dev):
        m = torch.nn.Sequential(torch.nn.Linear(64, 96), torch.nn.LayerNorm(96), torch.nn.Linear(96, 8))
        return m.to(dev).to(torch.bfloat16)

    torch.manual_seed(0)
    mg = make(cuda)
    torch.manual_seed(0)
    mc = make("cpu")
    outs = []
    for m in (mg, mc):
        named = list(m.named_parameters())
        sp = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
        nd = lambda n: n.endswith("bias")  # noqa: E731
        if name == "lamb":
            opt = FusedLAMB(sp, lr=1e-2, weight_decay=0.01, no_decay=nd, space=sp)
        elif name == "adamw":
            opt = FusedAdam(sp, lr=1e-2, weight_decay=0.01, no_decay=nd, space=sp)
        else:
            opt = FusedSGD(sp, lr=1e-2, momentum=0.9, weight_decay=1e-4, space=sp)
        dev = next(m.parameters()).device
        for it in range(3):
            torch.manual_seed(100 + it)
            x = torch.randn(16, 64).to(dev).bfloat16()
            loss = m(x).float().pow(2).mean()
            loss.backward()
            opt.step()
            opt.zero_grad()
        outs.append(sp.shard_params.detach().float().cpu())
    assert _rel(outs[0], outs[1]) < 2e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_fused_lamb_large_tensors_match_cpu(cuda, dtype):
    """LAMB's 8-wide kernels over multi-segment tensors (3M weights: 367 full 8K segments and a
    partial one, every per-thread chunk of a segment used) against the CPU implementation."""
    from cloudtik_amd.train.optim import FlatParamSpace, FusedLAMB

    def make(dev):
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(1024, 2936), torch.nn.LayerNorm(2936), torch.nn.Linear(2936, 40))
        return m.to(dev).to(dtype)

    outs = []
    for dev in (cuda, "cpu"):
        m = make(dev)
        named = list(m.named_parameters())
        sp = FlatParamSpace([p for _, p in named], names=[n for n, _ in named])
        opt = FusedLAMB(sp, lr=1e-2, weight_decay=0.01, no_decay=lambda n: n.endswith("bias"), space=sp)
        for it in range(2):
            g = torch.Generator().manual_seed(7 + it)
            x = torch.randn(32, 1024, generator=g).to(dev).to(dtype)
            m(x).float().pow(2).mean().backward()
            opt.step()
            opt.zero_grad()
        outs.append(sp.shard_params.detach().float().cpu())
    assert _rel(outs[0], outs[1]) < (1e-5 if dtype == torch.float32 else 2e-2)


def test_fused_lamb_v8_kernels_subprocess():
    """The opt-in 8-wide LAMB kernels (CLOUDTIK_AMD_LAMB_V8=1, read once per process) pass the
    same large-tensor check in a child process."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, CLOUDTIK_AMD_LAMB_V8="1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", __file__, "-k", "fused_lamb_large_tensors_match_cpu",
                        "-p", "no:cacheprovider"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("C,HW", [(64, 56), (256, 14), (2048, 7)])
@pytest.mark.parametrize("res", [False, True])
def test_batchnorm_act(cuda, C, HW, res):
    torch.manual_seed(0)
    N = 8
    x = (torch.randn(N, C, HW, HW, device=cuda) * 2 + 0.5).bfloat16().contiguous(
        memory_format=torch.channels_last).requires_grad_()
    r = torch.randn(N, C, HW, HW, device=cuda).bfloat16().contiguous(
        memory_format=torch.channels_last).requires_grad_() if res else None
    g = (1 + 0.1 * torch.randn(C, device=cuda)).bfloat16().requires_grad_()
    b = (0.1 * torch.randn(C, device=cuda)).bfloat16().requires_grad_()
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y = ops.batch_norm_act(x, g, b, rm, rv, residual=r, relu=True, training=True)
    dy = torch.randn_like(y)
    y.backward(dy)
    ts = [t.detach().float().requires_grad_() for t in ((x, g, b, r) if res else (x, g, b))]
    rm2, rv2 = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    yr = torch.nn.functional.batch_norm(ts[0], rm2, rv2, ts[1], ts[2], True, 0.1, 1e-5)
    if res:
        yr = yr + ts[3]
    yr = torch.relu(yr)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(rm, rm2) < 1e-3 and _rel(rv, rv2) < 1e-3
    grads = [x.grad, g.grad, b.grad] + ([r.grad] if res else [])
    for a, t in zip(grads, ts):
        assert _rel(a, t.grad) < 2e-2


@pytest.mark.parametrize("HW", [112, 37])
@pytest.mark.parametrize("shift", [0.5, -1.0])      # -1.0: most activations ReLU to 0 -> many ties
@pytest.mark.parametrize("bwd_fuse", [False, True])  # maxpool3s2_bwd_bn_kernel (pool grad + BN sums)
def test_bn_relu_maxpool_stem(cuda, HW, shift, bwd_fuse, monkeypatch):
    """Fused ResNet stem (bn_apply_pool_kernel + maxpool3s2_bwd_kernel, or the one-pass pool
    gradient + BatchNorm-backward reduction) vs the unfused native BN + PyTorch max_pool2d on the
    same bf16 tensors, and vs an fp32 reference."""
    from cloudtik_amd.ops import functional as FN
    monkeypatch.setattr(FN, "_STEM_POOL_BN_FUSE", bwd_fuse)
    torch.manual_seed(1)
    N, C = 4, 64
    x0 = (torch.randn(N, C, HW, HW, device=cuda) + shift).bfloat16().contiguous(memory_format=torch.channels_last)
    g0 = (1 + 0.1 * torch.randn(C, device=cuda)).bfloat16()
    b0 = (0.1 * torch.randn(C, device=cuda)).bfloat16()
    outs = []
    for fused in (True, False):
        x, g, b = (t.clone().requires_grad_() for t in (x0, g0, b0))
        rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
        if fused:
            y = ops.batch_norm_relu_maxpool(x, g, b, rm, rv, training=True)
        else:
            y = torch.nn.functional.max_pool2d(ops.batch_norm_act(x, g, b, rm, rv, relu=True, training=True), 3, 2, 1)
        torch.manual_seed(2)
        dy = torch.randn_like(y)
        y.backward(dy)
        outs.append((y.detach(), x.grad, g.grad, b.grad, rm, rv))
    (yf, dxf, dgf, dbf, rmf, rvf), (yu, dxu, dgu, dbu, rmu, rvu) = outs
    assert yf.shape == (N, C, (HW - 1) // 2 + 1, (HW - 1) // 2 + 1) and yf.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(yf, yu)                                  # same stats, same rounding, same max
    assert torch.equal(rmf, rmu) and torch.equal(rvf, rvu)
    assert _rel(dxf, dxu) < 1e-2 and _rel(dgf, dgu) < 1e-2 and _rel(dbf, dbu) < 1e-2
    # fp32 reference
    xr, gr, br = (t.detach().float().requires_grad_() for t in (x0, g0, b0))
    yr = torch.nn.functional.max_pool2d(torch.relu(torch.nn.functional.batch_norm(
        xr, torch.zeros(C, device=cuda), torch.ones(C, device=cuda), gr, br, True, 0.1, 1e-5)), 3, 2, 1)
    yr.backward(dy.float())
    assert _rel(yf, yr) < 1e-2
    if shift > 0:
        # with most activations ReLU'd to 0 the window maxima are near-ties whose winner
        # differs between bf16 and fp32 activations, so the gradient routing is only
        # comparable (exactly, above) against the same bf16 tensors
        assert _rel(dxf, xr.grad) < 3e-2 and _rel(dgf, gr.grad) < 3e-2


def test_deferred_conv_grads_match_preset(cuda):
    """FlatParamSpace(defer_conv_grads): conv-weight gradients taken from autograd and added
    into the flat buffer by one multi-tensor kernel (mt_add_) give the same flat gradient and
    the same SGD trajectory as preset .grad views, across gradient accumulation."""
    from cloudtik_amd.train.optim import FlatParamSpace, FusedSGD

    def make():
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Conv2d(16, 32, 3, padding=1, bias=False), torch.nn.ReLU(),
                                torch.nn.Conv2d(32, 32, 1, bias=False), torch.nn.Flatten(),
                                torch.nn.Linear(32 * 8 * 8, 10)).to(cuda).bfloat16()
        return m.to(memory_format=torch.channels_last)

    results = []
    for defer in (False, True):
        m = make()
        sp = FlatParamSpace(list(m.parameters()), defer_conv_grads=defer)
        opt = FusedSGD(sp.params, lr=0.05, momentum=0.9, space=sp)
        convs = [p for p in sp.params if p.dim() == 4]
        assert all((p.grad is None) == defer for p in convs)
        for step in range(3):
            for micro in range(2):                       # accumulation: second backward adds
                torch.manual_seed(10 * step + micro)
                x = torch.randn(8, 16, 8, 8, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
                m(x).float().pow(2).mean().backward()
            if step == 0:
                sp.flush_grads()
                results.append(sp.grad.detach().float().clone())
            opt.step()
            opt.zero_grad()
            assert not defer or all(p.grad is None for p in convs)
        results.append(sp.model.detach().float().clone())
    g0, w0, g1, w1 = results
    assert torch.allclose(g0, g1, rtol=1e-2, atol=1e-3)
    assert torch.allclose(w0, w1, rtol=1e-2, atol=1e-3)


def test_conv1x1_gemm_bottleneck(cuda, monkeypatch):
    """ResNet bottlenecks with the 1x1 convs as NHWC GEMMs and the residual / downsample
    gradient folded into conv1's dgrad GEMM (ops/conv1x1.py) match the stock MIOpen convs:
    output, input gradient and every parameter gradient, for a stage-1-like block (64-channel
    input: MIOpen dgrad) and a wide block (GEMM fwd + dgrad)."""
    from cloudtik_amd.models.resnet import Bottleneck
    from cloudtik_amd.ops import conv1x1 as C1

    def run(enabled, cin, width, down, H):
        monkeypatch.setattr(C1, "_ENABLED", enabled)
        torch.manual_seed(0)
        b = Bottleneck(cin, width, downsample=down, device=cuda, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        with torch.no_grad():
            for m in b.modules():
                if type(m).__name__ == "BatchNormAct":
                    m.weight.fill_(0.7)             # bn3's zero-init would hide the main branch
        x = torch.randn(8, cin, H, H, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
        x.requires_grad_()
        y = b(x)
        g = torch.randn_like(y)
        y.backward(g)
        return [y.float(), x.grad.float()] + [p.grad.float() for p in b.parameters()]

    for cin, width, down, H in ((64, 64, True, 14), (1024, 256, False, 7), (256, 128, True, 14)):
        ref, got = run(False, cin, width, down, H), run(True, cin, width, down, H)
        for a, b_ in zip(ref, got):
            assert _rel(b_, a) < 2e-2, (cin, width, down)


def test_conv_wgrad_side_stream_flat_buffer(cuda, monkeypatch):
    """Conv weight gradients computed on the gradient side stream and added straight into the
    flat buffer (ops/conv1x1.py _weight_grad) equal the AccumulateGrad / deferred path, across
    two accumulated backwards, and the bucketer callback fires once per weight."""
    from cloudtik_amd.models.resnet import Bottleneck
    from cloudtik_amd.ops import conv1x1 as C1
    from cloudtik_amd.ops.linear import sync_grad_stream
    from cloudtik_amd.train.optim import FlatParamSpace

    out = []
    for side in (False, True):
        monkeypatch.setattr(C1, "_SIDE_WGRAD", side)
        torch.manual_seed(0)
        b = Bottleneck(256, 128, downsample=True, device=cuda, dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        with torch.no_grad():
            b.bn3.weight.fill_(0.5)
        sp = FlatParamSpace(list(b.parameters()))
        calls = []
        for p in sp.params:
            p._ct_grad_ready = lambda p, calls=calls: calls.append(id(p))
        for micro in range(2):
            torch.manual_seed(1 + micro)
            x = torch.randn(16, 256, 14, 14, device=cuda).bfloat16().contiguous(memory_format=torch.channels_last)
            b(x).float().pow(2).mean().backward()
        sp.flush_grads()
        sync_grad_stream()
        torch.cuda.synchronize()
        out.append(sp.grad.float().clone())
        if side:       # conv1, conv2, conv3 (down is a plain nn.Conv2d here: stride 1 -> conv1x1 too)
            assert len(calls) >= 2 * 3
    assert _rel(out[1], out[0]) < 1e-2


def test_linear_fused_wgrad(cuda):
    from cloudtik_amd.train.optim import FlatParamSpace
    torch.manual_seed(0)
    lin = torch.nn.Linear(256, 512, device=cuda, dtype=torch.bfloat16)
    sp = FlatParamSpace([lin.weight, lin.bias], names=["w", "b"])
    seen = []
    lin.weight._ct_grad_ready = lambda p: seen.append(p)
    x = torch.randn(4, 33, 256, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    y = ops.linear(x, lin.weight, lin.bias)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, lin.weight, lin.bias))
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(dy.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(lin.weight.grad, wr.grad) < 1e-2
    assert _rel(lin.bias.grad, br.grad) < 1e-2
    assert len(seen) == 1
    # the weight grad must live in the flat buffer
    idx = [i for i, q in enumerate(sp.params) if q is lin.weight][0]
    assert lin.weight.grad.data_ptr() == sp.grad[sp.offsets[idx]:].data_ptr()


@pytest.mark.parametrize("N,K", [(1024, 1024), (3072, 1024), (512, 768)])
def test_wgrad_splitk_accumulate(cuda, N, K):
    from cloudtik_amd.ops.linear import splitk_factor, wgrad_accumulate
    T = 16384
    assert splitk_factor(T, N, K) > 1
    torch.manual_seed(0)
    dy = torch.randn(T, N, device=cuda, dtype=torch.bfloat16)
    x = torch.randn(T, K, device=cuda, dtype=torch.bfloat16)
    g0 = torch.randn(N, K, device=cuda, dtype=torch.bfloat16)
    g = g0.clone()
    wgrad_accumulate(g, dy, x)
    ref = g0.float() + dy.float().t() @ x.float()
    assert _rel(g, ref) < 5e-3
    # the non-split path agrees too
    g2 = g0.clone()
    g2.addmm_(dy.t(), x)
    assert _rel(g2, ref) < 5e-3


@pytest.mark.parametrize("p,fused,fused_fwd,stream", [(0.0, False, False, False), (0.1, False, False, False),
                                                     (0.1, True, False, False), (0.1, False, True, False),
                                                     (0.1, True, True, False), (0.1, True, True, True),
                                                     (0.1, True, True, "onetile")])
def test_bert_layer_blocks_match_composed(cuda, p, fused, fused_fwd, stream, monkeypatch):
    """Hand-scheduled block backward == composed-op autograd (same dropout streams); `fused`
    routes the FFN dgrad through the MFMA GEMM with the dGELU + bias-gradient epilogue,
    `fused_fwd` the FFN1 forward through it with the bias + GELU epilogue (the kept
    pre-activation then already holds the bias)."""
    from cloudtik_amd.models.bert import BertConfig, BertLayer
    from cloudtik_amd.ops import transformer as T
    monkeypatch.setattr(T, "_FUSED_FFN_DGRAD", fused)
    monkeypatch.setattr(T, "_FUSED_FFN_FWD", fused_fwd)
    stream_sites = []
    if stream:                             # every plain fwd / dgrad GEMM through an in-tree kernel
        sites = {"qkv", "wo", "ffn2", "do", "dx_attn", "dx_ffn"}
        monkeypatch.setattr(T, "_STREAM_SITES", set() if stream == "onetile" else sites)
        monkeypatch.setattr(T, "_ONETILE_SITES", sites if stream == "onetile" else set())
        orig_stream = T._stream_mm
        def spy_stream(site, *a, **k):
            r = orig_stream(site, *a, **k)
            if r is not None:
                stream_sites.append(site)
            return r
        monkeypatch.setattr(T, "_stream_mm", spy_stream)
    if fused_fwd:
        fwd_calls = []
        orig_fwd = T._fused_ffn1
        def spy_fwd(*a):
            r = orig_fwd(*a)
            fwd_calls.append(r is not None)
            return r
        monkeypatch.setattr(T, "_fused_ffn1", spy_fwd)
    if fused:
        calls = []
        orig_fused = T._fused_ffn_dgrad
        def spy(*a):
            r = orig_fused(*a)
            calls.append(r is not None)
            return r
        monkeypatch.setattr(T, "_fused_ffn_dgrad", spy)
    from cloudtik_amd.train.optim import FlatParamSpace
    cfg = BertConfig.tiny(hidden_size=256, num_attention_heads=4, intermediate_size=1024,
                          hidden_dropout_prob=p, attention_probs_dropout_prob=p)
    torch.manual_seed(0)
    lay = BertLayer(cfg, device=cuda, dtype=torch.bfloat16)
    named = list(lay.named_parameters())
    sp = FlatParamSpace([q for _, q in named], names=[n for n, _ in named])
    x = torch.randn(4, 64, 256, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    kb = torch.zeros(4, 64, device=cuda)
    kb[1, 50:] = -10000.0
    dy = torch.randn(4, 64, 256, device=cuda, dtype=torch.bfloat16)
    ops.manual_seed(5)
    y = lay(x, kb)
    y.backward(dy)
    g_blocks = sp.grad.clone().float()
    gx_blocks = x.grad.clone()
    # composed path (disable blocks)
    from cloudtik_amd.ops import transformer as T
    orig = T.blocks_supported
    T.blocks_supported = lambda *a, **k: False
    try:
        sp.zero_grad()
        x.grad = None
        ops.manual_seed(5)
        y2 = lay(x, kb)
        y2.backward(dy)
    finally:
        T.blocks_supported = orig
    assert _rel(y, y2) < 1e-2
    assert _rel(gx_blocks, x.grad) < 2e-2
    assert _rel(g_blocks, sp.grad.float()) < 2e-2
    if fused:
        assert calls and all(calls), "fused FFN dgrad path not taken"
    if fused_fwd:
        assert fwd_calls and all(fwd_calls), "fused FFN1 forward path not taken"
    if stream:
        assert set(stream_sites) == {"qkv", "wo", "ffn2", "do", "dx_attn", "dx_ffn"}, stream_sites


@pytest.mark.parametrize("name", ["adamw", "lamb"])
def test_optimizer_step_scalars_under_cpu_run_ahead(cuda, name):
    """The CPU queues several optimizer steps behind a long GPU kernel without synchronising:
    each step must still see ITS OWN lr / bias-correction factors (the per-step scalars are
    staged through pinned host memory that an async copy reads only when it executes)."""
    from cloudtik_amd.train.optim import FlatParamSpace, FusedAdam, FusedLAMB
    torch.manual_seed(0)
    w0 = torch.randn(4096, device=cuda)
    p = torch.nn.Parameter(w0.clone())
    sp = FlatParamSpace([p], names=["w"])
    kw = dict(lr=1e-2, weight_decay=0.01, space=sp)
    opt = FusedAdam(sp, **kw) if name == "adamw" else FusedLAMB(sp, bias_correction=True, **kw)
    lrs = [1e-2, 3e-2, 5e-3, 2e-2]
    grads = [torch.randn(4096, device=cuda) for _ in lrs]
    torch.cuda.synchronize()
    for lr, g in zip(lrs, grads):
        torch.cuda._sleep(20_000_000)            # keep the GPU busy so the CPU runs ahead
        for grp in opt.param_groups:
            grp["lr"] = lr
        sp.grad[:4096].copy_(g)
        opt.step()
    torch.cuda.synchronize()
    # fp32 reference of the same update rule, step by step
    w = w0.double().cpu()
    m = torch.zeros_like(w)
    v = torch.zeros_like(w)
    b1, b2, eps = 0.9, 0.999, opt.eps
    for t, (lr, g) in enumerate(zip(lrs, grads), 1):
        g = g.double().cpu()
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        u = (m / (1 - b1 ** t)) / ((v / (1 - b2 ** t)).sqrt() + eps) + 0.01 * w
        if name == "lamb":
            u = u * (w.norm() / u.norm())
        w = w - lr * u
    assert _rel(p.detach().double().cpu(), w) < 1e-5


@pytest.mark.parametrize("C", [64, 1024])
def test_batchnorm_repeat_and_relu_modes(cuda, C):
    """Back-to-back calls of different sizes are independent (same input -> same output), and
    the no-residual backward (ReLU mask recomputed from x and the forward's affine
    coefficients) matches the backward that reads the mask from y, bit for bit."""
    torch.manual_seed(1)
    C_ = ops.require_native()
    xa, xb = [(torch.randn(n, C, 7, 7, device=cuda) * 1.5 + 0.3).bfloat16().contiguous(
        memory_format=torch.channels_last) for n in (4, 16)]
    xs = [xa, xb, xa]
    g = (1 + 0.1 * torch.randn(C, device=cuda)).bfloat16()
    b = (0.1 * torch.randn(C, device=cuda)).bfloat16()
    outs = []
    for x in xs:
        rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
        y, stat = C_.bn_fwd_train(x, None, g, b, rm, rv, 1e-5, 0.1, True)
        dy = torch.randn_like(y, generator=None)
        d2 = C_.bn_bwd(dy, None, x, g, stat, 2, False, None, None)
        d1 = C_.bn_bwd(dy, y, x, g, stat, 1, False, None, None)
        assert torch.equal(d1[0], d2[0]) and torch.equal(d1[2], d2[2]) and torch.equal(d1[3], d2[3])
        # with a residual: the forward's ReLU bitmask (mode 3) == reading y (mode 1), bit for bit
        res = torch.randn_like(x)
        mask = torch.empty(x.numel() // 8, device=cuda, dtype=torch.uint8)
        yr, statr = C_.bn_fwd_train(x, res, g, b, rm.clone(), rv.clone(), 1e-5, 0.1, True, mask)
        assert torch.equal(mask.view(-1, 1).bitwise_and(1 << torch.arange(8, device=cuda, dtype=torch.uint8)) != 0,
                           (yr.permute(0, 2, 3, 1).reshape(-1, 8) > 0))
        m1 = C_.bn_bwd(dy, yr, x, g, statr, 1, True, None, None)
        m3 = C_.bn_bwd(dy, mask, x, g, statr, 3, True, None, None)
        for a_, b_ in zip(m1, m3):
            assert torch.equal(a_, b_)
        outs.append((y, stat, rm.clone()))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[2][0]) and torch.equal(outs[0][1], outs[2][1])
    ref_mean = xs[1].float().mean(dim=(0, 2, 3))
    assert _rel(outs[1][1][:C], ref_mean) < 1e-4


@pytest.mark.parametrize("V,ld", [(1000, 1024), (30522, 30720), (12000, 12000), (40000, 40000)])
@pytest.mark.parametrize("smooth", [0.0, 0.1])
def test_xent_kernel_matches_fp32(cuda, V, ld, smooth):
    """xent_fwd (in place, gradient written over the logits): loss rows, log-sum-exp and
    (softmax - onehot) * scale against an fp32 reference, padded columns zero.  Rows up to 32768
    columns run the register-resident kernel (one read of the row), wider rows the two-pass one
    (40000)."""
    from cloudtik_amd import ops as _ops
    C = _ops.require_native()
    torch.manual_seed(1)
    R = 37
    logits = (3 * torch.randn(R, ld, device=cuda)).bfloat16()
    labels = torch.randint(0, V, (R,), device=cuda)
    labels[::5] = -100
    labels[1] = V - 1                                   # the last real column
    ref = logits.float()[:, :V]
    lse_ref = torch.logsumexp(ref, 1)
    valid = labels != -100
    scale = torch.tensor([1.0 / valid.sum().item()], device=cuda)
    buf = logits.clone()
    loss, lse = C.xent_fwd(buf, buf, V, labels, scale, -100, smooth)
    torch.cuda.synchronize()
    logp = ref - lse_ref[:, None]
    nll = -logp.gather(1, labels.clamp_min(0)[:, None])[:, 0]
    want_loss = torch.where(valid, (1 - smooth) * nll - smooth * logp.mean(1), torch.zeros_like(nll))
    torch.testing.assert_close(lse, lse_ref, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(loss, want_loss, rtol=1e-3, atol=2e-3)
    onehot = torch.nn.functional.one_hot(labels.clamp_min(0), V).float()
    g = (logp.exp() - smooth / V - (1 - smooth) * onehot) * scale * valid[:, None].float()
    torch.testing.assert_close(buf.float()[:, :V], g, rtol=2e-2, atol=2e-4)
    assert buf.float()[:, V:].abs().max().item() == 0.0 if ld > V else True


def test_splitk_reduce2_matches_two_reductions(cuda):
    """One launch reducing a weight gradient's fp32 slabs and its bias partials (+= into bf16)."""
    torch.manual_seed(3)
    C = ops.require_native()
    P1 = torch.randn(5, 384, 256, device=cuda)
    P2 = torch.randn(5, 384, device=cuda)
    g1 = torch.randn(384, 256, device=cuda).bfloat16()
    g2 = torch.randn(384, device=cuda).bfloat16()
    r1 = (g1.float() + P1.sum(0)).bfloat16()
    r2 = (g2.float() + P2.sum(0)).bfloat16()
    C.splitk_reduce2(P1, g1, P2, g2, True)
    assert _rel(g1, r1) < 1e-2 and _rel(g2, r2) < 1e-2


@pytest.mark.parametrize("n", [4096, 3 * 2**20 + 64])
def test_sumsq_into_matches_torch(cuda, n):
    """Grad-norm clipping's sum of squares: per-block partials + one finishing block, added
    (+=) into the output."""
    torch.manual_seed(5)
    C = ops.require_native()
    x = torch.randn(n, device=cuda).bfloat16()
    out = torch.full((1,), 2.0, device=cuda)
    C.sumsq_into(x, out)
    ref = 2.0 + (x.float() ** 2).sum().item()
    assert abs(out.item() - ref) <= 1e-4 * ref


@pytest.mark.gpu
@pytest.mark.parametrize("C,tiles", [(64, 700), (128, 300), (256, 400), (192, 1000), (512, 130)])
def test_bn_bwd_given_many_tile_partials(cuda, C, tiles):
    """bn_bwd_given from producer per-tile sums (the conv data-gradient epilogue's): above the
    direct-finalize limit the first-level partials sum (batchnorm.hip bn_bwd_partials_sum_kernel,
    several tile rows per block below 256 channels) runs first.  dgamma / dbeta = column sums of
    the partials, dx = the closed form, against fp32."""
    torch.manual_seed(C + tiles)
    N, H = 2, 16
    x = torch.randn(N, C, H, H, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dym = torch.randn(N, C, H, H, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    mean = torch.randn(C, device=cuda) * 0.1
    invstd = torch.rand(C, device=cuda) + 0.5
    stat = torch.cat([mean, invstd, torch.zeros(2 * C, device=cuda)])
    gamma = (torch.rand(C, device=cuda) + 0.5).to(torch.bfloat16)
    p1 = torch.randn(tiles, C, device=cuda)
    p2 = torch.randn(tiles, C, device=cuda)
    part = torch.cat([p1.reshape(-1), p2.reshape(-1)])
    dx, dg, db = ops.require_native().bn_bwd_given(dym, x, gamma, stat, part, tiles, tiles, None, None)
    sdy, sdx = p1.sum(0), p2.sum(0)
    torch.testing.assert_close(db.float(), sdy, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(dg.float(), sdx, rtol=2e-2, atol=5e-2)
    M = N * H * H
    a = gamma.float() * invstd
    v = lambda t: t.view(1, -1, 1, 1)  # noqa: E731
    ref_dx = v(a) * dym.float() - v(a * sdx / M * invstd) * (x.float() - v(mean)) - v(a * sdy / M)
    assert ((dx.float() - ref_dx).norm() / ref_dx.norm()).item() < 1e-2
