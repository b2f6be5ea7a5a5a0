"""Hand-written MFMA GEMM D = A @ B^T (csrc/gemm_nt.hip) and its fused epilogues against
fp32 PyTorch references: plain / accumulate, bias + erf-GELU with the pre-activation kept,
dGELU with bias-gradient column sums; K-tile counts 1, 2, 3 and 16 exercise the prologue,
the steady-state DMA schedule and the drain; unsupported shapes are refused."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from cloudtik_amd import ops
    return ops.require_native()


def _gelu(x):
    return 0.5 * x * (1 + torch.erf(x / math.sqrt(2)))


def _gelu_grad(x):
    return 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(*shape, device="cuda", generator=g) * scale).to(torch.bfloat16)


def _close(out, ref, tol=2e-2):
    err = (out.float() - ref).abs().max().item()
    assert err <= tol * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 256, 128), (256, 768, 192), (2048, 1024, 1024)])
def test_gemm_nt_plain_and_accumulate(M, N, K):
    C = _C()
    A, B = _rand(M, K, seed=1), _rand(N, K, scale=K ** -0.5, seed=2)
    D = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nt(A, B, D, 0, False, None, None, None)
    ref = A.float() @ B.float().t()
    _close(D, ref)
    base = _rand(M, N, seed=3)
    D2 = base.clone()
    assert C.gemm_nt(A, B, D2, 0, True, None, None, None)
    _close(D2, ref + base.float())


def test_gemm_nt_bias_gelu_aux():
    C = _C()
    M, N, K = 1024, 512, 256
    A, B, bias = _rand(M, K, seed=4), _rand(N, K, scale=K ** -0.5, seed=5), _rand(N, scale=0.5, seed=6)
    h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.empty_like(h)
    assert C.gemm_nt(A, B, h, 1, False, bias, aux, None)
    z = A.float() @ B.float().t() + bias.float()
    _close(aux, z)
    _close(h, _gelu(z))


def test_gemm_nt_bias_gelu_stores_derivative():
    """EPI 6: h = gelu(z), aux = gelu'(z) (the FFN1 forward's derivative-storing epilogue)."""
    C = _C()
    M, N, K = 1024, 512, 256
    A, B, bias = _rand(M, K, seed=14), _rand(N, K, scale=K ** -0.5, seed=15), _rand(N, scale=0.5, seed=16)
    h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    g = torch.empty_like(h)
    assert C.gemm_nt(A, B, h, 6, False, bias, g, None)
    z = A.float() @ B.float().t() + bias.float()
    _close(h, _gelu(z))
    _close(g, _gelu_grad(z))
    assert (g.float() - _gelu_grad(z)).abs().max().item() < 1.5e-2     # bf16 rounding of values <= 1.13


@pytest.mark.parametrize("b_kn", [False, True])
def test_gemm_mul_aux_bgrad(b_kn):
    """EPI 7: dz = (A . B) * aux, dbias += column sums (the FFN data gradient with the stored
    gelu'), both operand layouts; agrees with EPI 2 on the same pre-activation."""
    C = _C()
    M, N, K = 1024, 768, 320
    A = _rand(M, K, seed=17)
    B = _rand(K, N, seed=18, scale=K ** -0.5) if b_kn else _rand(N, K, seed=18, scale=K ** -0.5)
    mm = C.gemm_nn if b_kn else C.gemm_nt
    ref_ab = A.float() @ (B.float() if b_kn else B.float().t())
    z = _rand(M, N, seed=19)
    g = _gelu_grad(z.float()).to(torch.bfloat16)
    dz = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    db = torch.full((N,), -0.5, device="cuda", dtype=torch.float32)
    assert mm(A, B, dz, 7, False, None, g, db)
    ref = ref_ab * g.float()
    _close(dz, ref)
    torch.testing.assert_close(db, ref.sum(0) - 0.5, rtol=2e-3, atol=2e-2 * max(1.0, ref.abs().sum(0).max().item() / M))
    dz2 = torch.empty_like(dz)
    assert mm(A, B, dz2, 2, False, None, z, None)                       # the recomputing epilogue
    assert (dz.float() - dz2.float()).abs().max().item() <= 2e-2 * max(1.0, ref.abs().max().item())


def test_gemm_nt_dgelu_bgrad():
    C = _C()
    M, N, K = 1024, 512, 320
    A, B = _rand(M, K, seed=7), _rand(N, K, scale=K ** -0.5, seed=8)
    aux = _rand(M, N, seed=9)
    dz = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    db = torch.full((N,), 0.25, device="cuda", dtype=torch.float32)      # accumulates into existing
    assert C.gemm_nt(A, B, dz, 2, False, None, aux, db)
    ref = (A.float() @ B.float().t()) * _gelu_grad(aux.float())
    _close(dz, ref)
    torch.testing.assert_close(db, ref.sum(0) + 0.25, rtol=2e-3, atol=2e-2)
    dz2 = torch.empty_like(dz)
    assert C.gemm_nt(A, B, dz2, 2, False, None, aux, None)               # no bias gradient
    assert torch.equal(dz, dz2)
    # pre-activation = aux + bias (aux saved without the bias, as the FFN block does)
    bias = _rand(N, scale=0.5, seed=12)
    db3 = torch.zeros(N, device="cuda", dtype=torch.float32)
    assert C.gemm_nt(A, B, dz2, 2, False, bias, aux, db3)
    ref3 = (A.float() @ B.float().t()) * _gelu_grad(aux.float() + bias.float())
    _close(dz2, ref3)
    torch.testing.assert_close(db3, ref3.sum(0), rtol=2e-3, atol=2e-2)


def test_gemm_nt_strided_operands_and_refusals():
    C = _C()
    big = _rand(512, 384, seed=10)
    A = big[:, :256]                      # lda = 384
    B = _rand(256, 256, seed=11)
    D = torch.empty(512, 256, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nt(A, B, D, 0, False, None, None, None)
    _close(D, A.float() @ B.float().t())
    Dw = torch.zeros(512, 384, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nt(A, B, Dw[:, 64:320], 0, False, None, None, None)            # ldd = 384, offset
    _close(Dw[:, 64:320], A.float() @ B.float().t())
    assert not Dw[:, :64].any() and not Dw[:, 320:].any()                       # nothing outside D
    bad = torch.empty(500, 256, device="cuda", dtype=torch.bfloat16)
    assert not C.gemm_nt(_rand(500, 256), B, bad, 0, False, None, None, None)     # M % 256
    assert not C.gemm_nt(_rand(256, 96), _rand(256, 96), torch.empty(256, 256, device="cuda",
                                                                      dtype=torch.bfloat16), 0, False, None, None,
                         None)                                                     # K % 64


def test_gemm_nt_operands_spanning_4gb_addresses():
    """Operand rows whose addresses span > 2^32 bytes (the staging addresses are split into a
    wave-uniform 64-bit base + a 32-bit lane offset: a sign-extension bug would fault here)."""
    C = _C()
    big = torch.empty(5 * 2 ** 30 // 2, device="cuda", dtype=torch.bfloat16)     # 5 GiB
    M, N, K = 512, 256, 2 ** 22                                                   # rows 8 MiB apart:
    A2 = big[: M * K].view(M, K)[:, :256]                                         # 4 GiB of addresses
    B = _rand(N, 256, seed=13)
    A2.copy_(_rand(M, 256, seed=14))
    D = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nt(A2, B, D, 0, False, None, None, None)
    _close(D, A2.float() @ B.float().t())
    del A2, big


def _split_ranges(K, S):
    """K range of each split-K slice: the K / 64 K-tiles dealt out, the first (K/64) % S
    slices one K-tile longer (ct_gemm_tn2)."""
    q, r = divmod(K // 64, S)
    out, k = [], 0
    for s in range(S):
        n = (q + (1 if s < r else 0)) * 64
        out.append((k, k + n))
        k += n
    return out


# ---- weight-gradient layout (ct_gemm_tn2): out = A[K,M]^T B[K,N], token-major operands
@pytest.mark.parametrize("M,N,K,S", [(256, 256, 64, 1), (512, 256, 128, 1), (256, 768, 192, 1),
                                     (768, 512, 1024, 1), (256, 256, 512, 8), (512, 768, 2048, 4),
                                     (1024, 256, 768, 3), (768, 256, 320, 3), (512, 512, 2048, 5),
                                     (256, 256, 192, 3)])
def test_gemm_tn2_matches_fp32(M, N, K, S):
    C = _C()
    A, B = _rand(K, M, seed=M + K), _rand(K, N, seed=N + 7 * K, scale=K ** -0.5)
    ref = A.float().t() @ B.float()
    if S == 1:
        D = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        assert C.gemm_tn2(A, B, D, 1, False)
        _close(D, ref)
        D0 = _rand(M, N, seed=3)
        D1 = D0.clone()
        assert C.gemm_tn2(A, B, D1, 1, True)
        _close(D1, ref + D0.float())
    else:
        P = torch.full((S, M, N), float("nan"), device="cuda")
        assert C.gemm_tn2(A, B, P, S, False)
        torch.testing.assert_close(P.sum(0), ref, rtol=2e-3, atol=2e-3 * ref.abs().max().item())
        # each slab is its own K range (uneven when S does not divide the K-tile count)
        for s_, (k0, k1) in enumerate(_split_ranges(K, S)):
            torch.testing.assert_close(P[s_], A[k0:k1].float().t() @ B[k0:k1].float(), rtol=2e-3,
                                       atol=2e-3 * ref.abs().max().item())


def test_gemm_tn2_strided_operands_and_refusals():
    C = _C()
    big = _rand(256, 640, seed=21)
    A = big[:, 128:384]                  # lda = 640, column offset
    B = _rand(256, 512, seed=22)
    D = torch.zeros(256, 768, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_tn2(A, B, D[:, 128:640], 1, False)                       # ldo = 768
    _close(D[:, 128:640], A.float().t() @ B.float())
    assert not D[:, :128].any() and not D[:, 640:].any()
    assert not C.gemm_tn2(_rand(96, 256), _rand(96, 256), torch.empty(256, 256, device="cuda",
                                                                      dtype=torch.bfloat16), 1, False)   # K % 64
    assert not C.gemm_tn2(_rand(128, 256), _rand(128, 256), torch.empty(3, 256, 256, device="cuda"), 3,
                          False)                                      # fewer K-tiles (2) than splits


# ---- NN layout (gemm_nn): D = A[M,K] @ B[K,N], B read in place from an [out, in] weight
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 192), (2048, 1024, 1024)])
def test_gemm_nn_plain_and_dgelu(M, N, K):
    C = _C()
    A, B = _rand(M, K, seed=M), _rand(K, N, seed=N, scale=K ** -0.5)
    ref = A.float() @ B.float()
    D = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nn(A, B, D, 0, False, None, None, None)
    _close(D, ref)
    aux = _rand(M, N, seed=5)
    bias = _rand(N, seed=6, scale=0.1)
    db = torch.zeros(N, device="cuda")
    assert C.gemm_nn(A, B, D, 2, False, bias, aux, db)
    want = ref * _gelu_grad(aux.float() + bias.float())
    _close(D, want)
    torch.testing.assert_close(db, want.sum(0), rtol=2e-3, atol=2e-2 * max(1.0, want.abs().sum(0).max().item() / M))
    # strided B (a column slice of a wider weight)
    Bw = _rand(K, N + 128, seed=7)
    assert C.gemm_nn(A, Bw[:, 128:], D, 0, False, None, None, None)
    _close(D, A.float() @ Bw[:, 128:].float())


@pytest.mark.parametrize("M,N,K,S", [(512, 256, 256, 1), (768, 512, 2048, 4), (3072, 1024, 8192, 16),
                                     (3072, 1024, 8192, 5)])
def test_gemm_tn2_bias_column_sums(M, N, K, S):
    """gemm_tn2_bias: the weight-gradient product plus per-split column sums of A (the bias
    gradient) from the extra all-ones MFMA; the product itself is unchanged."""
    C = _C()
    A, B = _rand(K, M, seed=M + 1), _rand(K, N, seed=N + 2, scale=K ** -0.5)
    ref = A.float().t() @ B.float()
    bP = torch.full((S, M), float("nan"), device="cuda")
    if S == 1:
        D = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        assert C.gemm_tn2_bias(A, B, D, 1, True, bP)
        _close(D, ref)
    else:
        P = torch.empty(S, M, N, device="cuda")
        assert C.gemm_tn2_bias(A, B, P, S, False, bP)
        torch.testing.assert_close(P.sum(0), ref, rtol=2e-3, atol=2e-3 * ref.abs().max().item())
    want = torch.stack([A[k0:k1].float().sum(0) for k0, k1 in _split_ranges(K, S)])
    torch.testing.assert_close(bP, want, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("M,N,K,wgs", [(256, 256, 64, 0), (512, 256, 128, 1), (1024, 768, 192, 5),
                                       (2048, 1024, 1024, 0), (1536, 512, 320, 3), (4096, 3072, 1024, 0)])
@pytest.mark.parametrize("b_kn", [False, True])
def test_gemm_nt_stream_matches_reference(M, N, K, wgs, b_kn):
    """Streamed persistent kernel: every workgroup walks several output tiles with one DMA
    stream (wgs < tiles forces several tiles per workgroup, including uneven tails and single
    K-tile streams); NT and NN (B stored [K, N]) layouts, with and without bias."""
    C = _C()
    A = _rand(M, K, seed=11)
    B = _rand(K, N, scale=K ** -0.5, seed=12) if b_kn else _rand(N, K, scale=K ** -0.5, seed=12)
    bias = _rand(N, scale=0.5, seed=13)
    ref = A.float() @ (B.float() if b_kn else B.float().t())
    D = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    assert C.gemm_nt_stream(A, B, D, None, b_kn, wgs)
    torch.cuda.synchronize()
    _close(D, ref)
    D.fill_(float("nan"))
    assert C.gemm_nt_stream(A, B, D, bias, b_kn, wgs)
    _close(D, ref + bias.float())
    base = _rand(M, N, seed=14)
    D2 = base.clone()
    assert C.gemm_nt_stream(A, B, D2, None, b_kn, wgs, True)            # D += A B
    _close(D2, ref + base.float())


def test_gemm_nt_stream_refuses_unsupported():
    C = _C()
    A, B = _rand(300, 64), _rand(256, 64)
    D = torch.empty(300, 256, device="cuda", dtype=torch.bfloat16)
    assert not C.gemm_nt_stream(A, B, D, None, False, 0)


@pytest.mark.parametrize("knob", ["CLOUDTIK_AMD_GEMM_STAGGER=-1", "CLOUDTIK_AMD_GEMM_GROUP_M=1"])
def test_gemm_staggered_grid_covers_every_tile_subprocess(knob):
    """The non-default tile orders -- the staggered grid (CLOUDTIK_AMD_GEMM_STAGGER=-1: 128 full /
    column-half pairs first, the other column halves last, on a >= 2-round grid) and the plain
    row-major order (CLOUDTIK_AMD_GEMM_GROUP_M=1; the default walks 4 M-tiles per N-tile) --
    still write every tile exactly once for every epilogue kind: the test below in a child
    process with the knob set (the library reads it once per process)."""
    import os
    import subprocess
    import sys
    k, v = knob.split("=")
    env = dict(os.environ, **{k: v})
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", __file__, "-k", "staggered_grid_covers_every_tile and not subprocess",
                        "-p", "no:cacheprovider"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]


@pytest.mark.parametrize("b_kn", [False, True])
def test_gemm_staggered_grid_covers_every_tile(b_kn):
    """>= 2 rounds of tiles (8192 x 4096: 512 tiles on 256 CUs); with the stagger on (the
    subprocess test above) 128 full / column-half pairs come first and the other column halves
    last.  Every epilogue kind must write every tile exactly once (plain, accumulate,
    bias-GELU + gelu', x gelu' + bias grad)."""
    C = _C()
    M, N, K = 8192, 4096, 128
    mm = C.gemm_nn if b_kn else C.gemm_nt
    A = _rand(M, K, seed=31)
    B = _rand(K, N, seed=32, scale=K ** -0.5) if b_kn else _rand(N, K, seed=32, scale=K ** -0.5)
    ref = A.float() @ (B.float() if b_kn else B.float().t())
    D = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    assert mm(A, B, D, 0, False, None, None, None)
    _close(D, ref)
    base = _rand(M, N, seed=33)
    D2 = base.clone()
    assert mm(A, B, D2, 0, True, None, None, None)
    _close(D2, ref + base.float())
    bias = _rand(N, scale=0.5, seed=34)
    h, g = torch.full_like(D, float("nan")), torch.full_like(D, float("nan"))
    assert mm(A, B, h, 6, False, bias, g, None)
    z = ref + bias.float()
    _close(h, _gelu(z))
    _close(g, _gelu_grad(z))
    db = torch.zeros(N, device="cuda", dtype=torch.float32)
    dz = torch.full_like(D, float("nan"))
    assert mm(A, B, dz, 7, False, None, g, db)
    want = ref * g.float()
    _close(dz, want)
    torch.testing.assert_close(db, want.sum(0), rtol=3e-3, atol=5e-2 * max(1.0, want.abs().sum(0).max().item() / M))
