"""Paired-tile persistent MFMA GEMM (ops/csrc/gemm_pp.hip) against fp32 PyTorch references:
D = A @ B^T with the plain, +bias and bias + erf-GELU (+ gelu' aux) epilogues, on shapes whose
128 x 256 tiles split unevenly over the two wave groups of every workgroup (the barrier-count
padding), several epilogue-slot splits, and the BERT-large FFN1 shape on the whole chip."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from cloudtik_amd import ops
    return ops.require_native()


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


@pytest.mark.parametrize("M,N,K,wgs", [(2048, 512, 256, 8), (2176, 768, 192, 8), (3968, 1280, 640, 16),
                                       (4096, 1024, 1024, 32)])
@pytest.mark.parametrize("epi", [0, 5, 6])
@pytest.mark.parametrize("eslots", [1, 4, 8])
def test_gemm_pp_matches_fp32(M, N, K, wgs, epi, eslots):
    C = _C()
    g = torch.Generator().manual_seed(M + N + K + epi)
    A = torch.randn(M, K, generator=g).cuda().bfloat16()
    B = (torch.randn(N, K, generator=g) * K ** -0.5).cuda().bfloat16()
    bias = (torch.randn(N, generator=g) * 0.5).cuda().bfloat16()
    D = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    aux = torch.full_like(D, float("nan")) if epi == 6 else None
    assert C.gemm_pp(A, B, D, epi, bias if epi else None, aux, wgs, eslots)
    torch.cuda.synchronize()
    z, d = _ref(A, B, bias, epi)
    assert not torch.isnan(D).any()                        # every tile written
    assert _rel(D, z) < 6e-3
    if epi == 6:
        assert not torch.isnan(aux).any() and _rel(aux, d) < 6e-3


def test_gemm_pp_full_chip_ffn1_shape_and_rejects():
    C = _C()
    g = torch.Generator().manual_seed(7)
    M, N, K = 32768, 4096, 1024
    A = torch.randn(M, K, generator=g).cuda().bfloat16()
    B = (torch.randn(N, K, generator=g) * K ** -0.5).cuda().bfloat16()
    bias = (torch.randn(N, generator=g) * 0.5).cuda().bfloat16()
    D = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.empty_like(D)
    assert C.gemm_pp(A, B, D, 6, bias, aux, 0, 4)
    z, d = _ref(A, B, bias, 6)
    assert _rel(D, z) < 6e-3 and _rel(aux, d) < 6e-3
    # unsupported: N % 256, K % 64, fewer tiles than virtual CTAs -> nothing launched
    assert not C.gemm_pp(A, B[:3968], torch.empty(M, 3968, device="cuda", dtype=torch.bfloat16), 0, None, None, 0, 4)
    assert not C.gemm_pp(A[:, :992].contiguous(), B[:, :992].contiguous(), D, 0, None, None, 0, 4)
    assert not C.gemm_pp(A[:1024], B, D[:1024], 0, None, None, 0, 4)
