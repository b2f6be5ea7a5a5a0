"""Four-wave MFMA GEMM (ops/csrc/gemm_nt.hip gemm_w4_kernel: 128 x 128 per wave, accumulators
pinned in AGPRs by inline-asm MFMAs) against fp32 PyTorch references: plain, +bias and
bias + erf-GELU (+ gelu' aux) epilogues, one to many K-tiles (the peeled first / last tiles)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(A, B, bias, epi):
    z = A.float() @ B.float().t()
    if epi == 0:
        return z, None
    z = z + bias.float()
    if epi == 5:
        return z, None
    phi = 0.5 * (1.0 + torch.erf(z / math.sqrt(2.0)))
    return z * phi, phi + z * torch.exp(-0.5 * z * z) / math.sqrt(2.0 * math.pi)


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 128), (768, 512, 192), (2048, 1024, 1024)])
@pytest.mark.parametrize("epi", [0, 5, 6])
def test_gemm_w4_matches_fp32(M, N, K, epi):
    from cloudtik_amd import ops
    C = ops.require_native()
    g = torch.Generator().manual_seed(M + N + K + epi)
    A = torch.randn(M, K, generator=g).cuda().bfloat16()
    B = (torch.randn(N, K, generator=g) * K ** -0.5).cuda().bfloat16()
    bias = (torch.randn(N, generator=g) * 0.5).cuda().bfloat16()
    D = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    aux = torch.full_like(D, float("nan")) if epi == 6 else None
    assert C.gemm_w4(A, B, D, epi, bias if epi else None, aux)
    torch.cuda.synchronize()
    z, d = _ref(A, B, bias, epi)
    assert not torch.isnan(D).any() and _rel(D, z) < 6e-3
    if epi == 6:
        assert not torch.isnan(aux).any() and _rel(aux, d) < 6e-3


def test_gemm_w4_rejects_unsupported_shapes():
    from cloudtik_amd import ops
    C = ops.require_native()
    A = torch.randn(512, 192, device="cuda").bfloat16()
    B = torch.randn(384, 192, device="cuda").bfloat16()              # N % 256
    assert not C.gemm_w4(A, B, torch.empty(512, 384, device="cuda", dtype=torch.bfloat16), 0)
    B = torch.randn(256, 160, device="cuda").bfloat16()              # K % 64
    assert not C.gemm_w4(A[:, :160].contiguous(), B, torch.empty(512, 256, device="cuda", dtype=torch.bfloat16), 0)
