"""GPU numerics of RoPE, EmbeddingBag / interaction, detection ops and multi-tensor copy,
each against a plain fp32 PyTorch reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


# ---------------------------------------------------------------------- RoPE
@pytest.mark.parametrize("neox", [True, False])
@pytest.mark.parametrize("with_pos", [False, True])
def test_rope_fwd_bwd(cuda, neox, with_pos):
    from cloudtik_amd.ops.rope import apply_rotary, rope_reference, rotary_cache
    torch.manual_seed(0)
    B, S, H, Hk, D = 3, 37, 4, 2, 64
    cos, sin = rotary_cache(128, D, device=cuda)
    q = torch.randn(B, S, H, D, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hk, D, device=cuda, dtype=torch.bfloat16, requires_grad=True)
    pos = torch.randint(0, 128, (B, S), device=cuda) if with_pos else None
    qo, ko = apply_rotary(q, k, cos, sin, pos, neox)
    p = pos.reshape(-1) if with_pos else torch.arange(B * S, device=cuda) % S
    qr = rope_reference(q.detach().reshape(-1, H, D), cos, sin, p, neox)
    kr = rope_reference(k.detach().reshape(-1, Hk, D), cos, sin, p, neox)
    assert _rel(qo.reshape(-1, H, D), qr) < 1e-2 and _rel(ko.reshape(-1, Hk, D), kr) < 1e-2
    gq, gk = torch.randn_like(qo), torch.randn_like(ko)
    (qo * gq).sum().add_((ko * gk).sum()).backward()
    # rotation is orthogonal: grad = inverse rotation of the upstream grad
    dq_ref = rope_reference(gq.reshape(-1, H, D), cos, sin, p, neox, inverse=True)
    dk_ref = rope_reference(gk.reshape(-1, Hk, D), cos, sin, p, neox, inverse=True)
    assert _rel(q.grad.reshape(-1, H, D), dq_ref) < 1e-2 and _rel(k.grad.reshape(-1, Hk, D), dk_ref) < 1e-2


def test_rope_strided_qkv_view(cuda):
    """q/k as views into a packed [T, 3, H, D] qkv tensor (no copy in the caller)."""
    from cloudtik_amd.ops.rope import rope_reference, rotary_cache
    from cloudtik_amd import ops
    T, H, D = 50, 4, 128
    cos, sin = rotary_cache(64, D, device=cuda)
    qkv = torch.randn(T, 3, H, D, device=cuda, dtype=torch.bfloat16)
    ref_q = rope_reference(qkv[:, 0], cos, sin, torch.arange(T, device=cuda) % 25, True)
    q, k = qkv[:, 0], qkv[:, 1]
    ops.require_native().rope(q, k, cos, sin, None, 25, True, False)
    assert _rel(qkv[:, 0], ref_q) < 1e-2


# ---------------------------------------------------------------------- EmbeddingBag
def _bags(T, B, V, maxlen, device, g):
    idx, offs = [], []
    for t in range(T):
        lens = torch.randint(0, maxlen + 1, (B,), generator=g)
        o = torch.zeros(B, dtype=torch.int64)
        o[1:] = lens.cumsum(0)[:-1]
        idx.append(torch.randint(0, V[t], (int(lens.sum()),), generator=g))
        offs.append(o)
    from cloudtik_amd.ops.embedding import pack_bags
    i, o = pack_bags(idx, offs, B)
    return i.to(device), o.to(device)


@pytest.mark.parametrize("mean", [False, True])
@pytest.mark.parametrize("with_psw", [False, True])
def test_embedding_bag(cuda, mean, with_psw):
    from cloudtik_amd.ops.embedding import EmbeddingBagCollection, embedding_bag_reference
    g = torch.Generator().manual_seed(1)
    V, E, B = [100, 37, 1000], 64, 33
    ebc = EmbeddingBagCollection(V, E, mode="mean" if mean else "sum", device=cuda)
    idx, offs = _bags(len(V), B, V, 5, cuda, g)
    psw = torch.rand(idx.numel(), device=cuda, requires_grad=True) if with_psw else None
    out = ebc(idx, offs, B, psw)
    W = ebc.weight.detach().clone().requires_grad_()
    pr = psw.detach().clone().requires_grad_() if with_psw else None
    ref = embedding_bag_reference(W, ebc.row_base, idx, offs, B, pr, mean)
    assert out.shape == (B, len(V), E) and _rel(out, ref) < 1e-5
    go = torch.randn_like(out)
    out.backward(go)
    ref.backward(go)
    assert _rel(ebc.weight.grad, W.grad) < 1e-5
    if with_psw:
        assert _rel(psw.grad, pr.grad) < 1e-4


def test_embedding_bag_fused_sgd(cuda):
    from cloudtik_amd.ops.embedding import EmbeddingBagCollection, embedding_bag_reference
    g = torch.Generator().manual_seed(2)
    V, E, B, lr = [50, 60], 128, 16, 0.5
    ebc = EmbeddingBagCollection(V, E, device=cuda, sparse_lr=lr)
    W0 = ebc.weight.detach().clone().requires_grad_()
    idx, offs = _bags(len(V), B, V, 4, cuda, g)
    out = ebc(idx, offs, B)
    go = torch.randn_like(out)
    out.backward(go)
    assert ebc.weight.grad is None            # applied in the backward kernel
    embedding_bag_reference(W0, ebc.row_base, idx, offs, B).backward(go)
    assert _rel(ebc.weight.detach(), W0.detach() - lr * W0.grad) < 1e-6


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_dot_interaction(cuda, dtype):
    from cloudtik_amd.ops.embedding import dot_interaction, interaction_reference
    torch.manual_seed(3)
    B, T, E = 37, 26, 64
    x = torch.randn(B, E, device=cuda, dtype=dtype, requires_grad=True)
    emb = torch.randn(B, T, E, device=cuda, dtype=dtype, requires_grad=True)
    out = dot_interaction(x, emb)
    xr, er = x.detach().float().requires_grad_(), emb.detach().float().requires_grad_()
    ref = interaction_reference(xr, er)
    assert out.shape == (B, E + 27 * 26 // 2)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(out, ref) < tol
    go = torch.randn_like(out)
    out.backward(go)
    ref.backward(go.float())
    assert _rel(x.grad, xr.grad) < tol and _rel(emb.grad, er.grad) < tol


# ---------------------------------------------------------------------- detection
@pytest.mark.parametrize("n", [1, 63, 700, 3000])
def test_nms_matches_reference(cuda, n):
    from cloudtik_amd.ops.vision import nms, nms_reference
    g = torch.Generator().manual_seed(n)
    xy = torch.rand(n, 2, generator=g) * 200
    wh = torch.rand(n, 2, generator=g) * 60 + 1
    boxes = torch.cat([xy, xy + wh], 1)
    scores = torch.rand(n, generator=g)
    ref = nms_reference(boxes, scores, 0.5)
    got = nms(boxes.to(cuda), scores.to(cuda), 0.5).cpu()
    assert torch.equal(got, ref)


def test_batched_nms_keeps_categories_apart(cuda):
    from cloudtik_amd.ops.vision import batched_nms
    boxes = torch.tensor([[0, 0, 10, 10], [0, 0, 10, 10], [1, 1, 10, 10.]], device=cuda)
    scores = torch.tensor([0.9, 0.8, 0.7], device=cuda)
    keep = batched_nms(boxes, scores, torch.tensor([0, 1, 0], device=cuda), 0.5)
    assert sorted(keep.tolist()) == [0, 1]


def _rois(K, N, H, W, g):
    b = torch.randint(0, N, (K, 1), generator=g).float()
    xy = torch.rand(K, 2, generator=g) * torch.tensor([W * 0.6, H * 0.6])
    wh = torch.rand(K, 2, generator=g) * torch.tensor([W * 0.4, H * 0.4]) + 0.5
    return torch.cat([b, xy, xy + wh], 1)


@pytest.mark.parametrize("aligned", [False, True])
@pytest.mark.parametrize("sr", [2, -1])
def test_roi_align(cuda, aligned, sr):
    from cloudtik_amd.ops.vision import roi_align, roi_align_reference
    g = torch.Generator().manual_seed(4)
    feat = torch.randn(2, 3, 12, 14, generator=g)
    rois = _rois(5, 2, 12, 14, g)
    fr = feat.clone().requires_grad_()
    ref = roi_align_reference(fr, rois, (4, 3), 1.0, sr, aligned)
    fg = feat.to(cuda).requires_grad_()
    out = roi_align(fg, rois.to(cuda), (4, 3), 1.0, sr, aligned)
    assert _rel(out.cpu(), ref) < 1e-5
    go = torch.randn_like(ref)
    ref.backward(go)
    out.backward(go.to(cuda))
    assert _rel(fg.grad.cpu(), fr.grad) < 1e-5


def test_roi_pool(cuda):
    from cloudtik_amd.ops.vision import roi_pool, roi_pool_reference
    g = torch.Generator().manual_seed(5)
    feat = torch.randn(2, 4, 16, 16, generator=g)
    rois = _rois(6, 2, 16, 16, g) * torch.tensor([1, 2, 2, 2, 2.])
    ref = roi_pool_reference(feat, rois, (3, 3), 0.5)
    fg = feat.to(cuda).requires_grad_()
    out = roi_pool(fg, rois.to(cuda), (3, 3), 0.5)
    assert _rel(out.cpu(), ref) < 1e-6
    out.sum().backward()
    assert abs(fg.grad.sum().item() - (ref != 0).float().sum().item()) < 1e-3


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sigmoid_focal_loss(cuda, dtype):
    from cloudtik_amd.ops.vision import sigmoid_focal_loss, sigmoid_focal_loss_reference
    g = torch.Generator().manual_seed(6)
    logits = (torch.randn(200, 9, generator=g) * 4).to(dtype)
    tgt = torch.randint(-1, 10, (200,), generator=g)
    lr = logits.float().clone().requires_grad_()
    ref = sigmoid_focal_loss_reference(lr, tgt, 2.0, 0.25)
    lg = logits.to(cuda).requires_grad_()
    out = sigmoid_focal_loss(lg, tgt.to(cuda), 2.0, 0.25, reduction="none")
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert _rel(out.cpu(), ref) < tol
    go = torch.rand_like(ref)
    ref.backward(go)
    out.backward(go.to(cuda))
    assert _rel(lg.grad.cpu(), lr.grad) < tol


# ---------------------------------------------------------------------- multi-tensor copy
@pytest.mark.parametrize("flat_dtype", [torch.float32, torch.bfloat16])
def test_multi_tensor_pack_unpack(cuda, flat_dtype):
    from cloudtik_amd.ops.multi_tensor import pack, unpack
    ts = [torch.randn(n, device=cuda) for n in (1, 1000, 77, 4096 * 3 + 5)]
    flat = pack(ts, scale=0.5, dtype=flat_dtype)
    ref = torch.cat([t.reshape(-1) for t in ts]) * 0.5
    assert _rel(flat, ref) < (1e-7 if flat_dtype == torch.float32 else 5e-3)
    outs = [torch.empty_like(t) for t in ts]
    unpack(flat, outs, scale=2.0)
    for a, b in zip(outs, ts):
        assert _rel(a, b) < (1e-7 if flat_dtype == torch.float32 else 5e-3)


@pytest.mark.gpu
def test_bn_grads_accumulate_into_flat_buffer(cuda):
    """BatchNorm parameter gradients written straight into the flat gradient buffer equal the
    autograd (AccumulateGrad) path, and the bucketer is notified for every parameter."""
    import copy
    from cloudtik_amd.models.resnet import ResNet
    from cloudtik_amd.train.optim import FlatParamSpace
    torch.manual_seed(0)
    a = ResNet((1, 1, 1, 1), 10, device=cuda, dtype=torch.bfloat16)
    b = copy.deepcopy(a)
    space = FlatParamSpace(list(b.parameters()))
    seen = []
    for p in space.params:
        p._ct_grad_ready = lambda p, seen=seen: seen.append(id(p))
        p.register_post_accumulate_grad_hook(lambda p, seen=seen: seen.append(id(p)))
    x = torch.randn(8, 3, 64, 64, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for m in (a, b):
        torch.nn.functional.cross_entropy(m(x).float(), torch.arange(8, device=cuda) % 10).backward()
    # conv weights: deferred (AccumulateGrad output flushed into the flat buffer) or written
    # into the flat buffer on the gradient side stream -- either way read the flat view
    from cloudtik_amd.ops.linear import sync_grad_stream
    sync_grad_stream()
    space.flush_grads()
    torch.cuda.synchronize()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        gb = pb.grad if pb.grad is not None else getattr(pb, "_ct_flat_view", None)
        assert gb is not None, n
        torch.testing.assert_close(gb.float(), pa.grad.float(), atol=2e-2, rtol=2e-2, msg=n)
    assert set(id(p) for p in space.params) <= set(seen)


@pytest.mark.parametrize("splits,acc", [(1, False), (1, True), (3, False)])
def test_gemm_tn_weight_gradient(cuda, splits, acc):
    """MFMA dW kernel (csrc/gemm_nt.hip, TN layout): C[M,N] (+)= A[T,M]^T B[T,N] vs an fp32
    reference, asymmetric operands (a row/col swap fails), split-K fp32 slabs and bf16
    accumulate; then the wgrad entry point (ops.linear.wgrad_accumulate) on the same data."""
    import importlib
    from cloudtik_amd import ops
    L = importlib.import_module("cloudtik_amd.ops.linear")     # (ops.linear is the function)
    C = ops.require_native()
    g = torch.Generator().manual_seed(3)
    T, M, N = 64 * 3 * 4, 512, 768
    A = (torch.randn(T, M, generator=g) + torch.arange(M) / M).bfloat16().to(cuda)
    B = (torch.randn(T, N, generator=g) - torch.arange(N)[None, :] / N).bfloat16().to(cuda)
    ref = A.float().t() @ B.float()
    if splits > 1:
        out = torch.empty(splits, M, N, device=cuda)
        assert C.gemm_tn2(A, B, out, splits, False)
        torch.testing.assert_close(out.sum(0), ref, atol=2e-3, rtol=1e-4)
    else:
        base = torch.randn(M, N, generator=g).bfloat16().to(cuda)
        out = base.clone()
        assert C.gemm_tn2(A, B, out, 1, acc)
        want = ref + (base.float() if acc else 0)
        torch.testing.assert_close(out.float(), want, atol=0.5, rtol=1e-2)
    # unsupported shapes are refused, not launched
    assert not C.gemm_tn2(A[:, :500], B, torch.empty(2, 500, N, device=cuda), 2, False)
    # the weight-gradient entry point accumulates the same product into a bf16 gradient
    grad = torch.randn(M, N, generator=g).bfloat16().to(cuda)
    want = ref + grad.float()
    L.wgrad_accumulate(grad, A, B)
    torch.testing.assert_close(grad.float(), want, atol=0.5, rtol=1e-2)
