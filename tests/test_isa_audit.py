"""Static audit of the compiled gfx950 kernels (scripts/isa_audit.py), on the CPU.

- The checker finds the hazards it is meant to find (crafted assembly).
- Every HIP source with inline-asm LDS-DMA is free of the readlane -> VMEM saddr hazard.
- The LayerNorm backward's two-row prefetch loop keeps its waits counted (no vmcnt(0) drain).
"""
import os
import shutil
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import isa_audit as A  # noqa: E402

needs_hipcc = pytest.mark.skipif(not (os.path.exists(A.HIPCC) or shutil.which("hipcc")), reason="no hipcc")


def test_readlane_vmem_hazard_detected_and_cleared_by_nops():
    bad = ["v_readfirstlane_b32 s4, v1", "v_readfirstlane_b32 s5, v2", "s_mov_b32 m0, s6",
           "global_load_lds_dwordx4 v3, s[4:5]"]
    found = A.readlane_vmem_hazards(bad)
    assert len(found) == 2 and all("s[4:5]" in f[2] for f in found)      # s4 and s5
    padded = bad[:3] + ["s_nop 4"] + bad[3:]
    assert A.readlane_vmem_hazards(padded) == []
    # an SGPR the VMEM does not read, and a read that is 5 instructions later, are fine
    assert A.readlane_vmem_hazards(["v_readlane_b32 s9, v1, 3", "global_load_dwordx4 v[0:3], v4, s[4:5]"]) == []
    far = ["v_readlane_b32 s4, v1, 0"] + ["v_add_u32 v7, v7, v8"] * 5 + ["buffer_load_dword v0, v1, s[0:3], s4 offen"]
    assert A.readlane_vmem_hazards(far) == []
    near = ["v_readlane_b32 s4, v1, 0"] + ["v_add_u32 v7, v7, v8"] * 3 + ["buffer_load_dword v0, v1, s[0:3], s4 offen"]
    assert len(A.readlane_vmem_hazards(near)) == 1


def test_loop_drain_detected():
    lines = [".LBB0_1:", "global_load_dwordx4 v[0:3], v[4:5], off", "s_waitcnt vmcnt(0)",
             "v_add_f32 v6, v0, v1", "s_cbranch_scc1 .LBB0_1", "s_waitcnt vmcnt(0)", "s_endpgm"]
    d = A.loop_drains(lines)
    assert d == [(".LBB0_1", 2)]                      # the wait after the loop is not reported
    counted = list(lines)
    counted[2] = "s_waitcnt vmcnt(2)"
    assert A.loop_drains(counted) == []


@needs_hipcc
def test_asm_dma_sources_have_no_readlane_vmem_hazard():
    srcs = [os.path.join(A.CSRC, f) for f in ("gemm_nt.hip", "gemm_pp.hip", "attention.hip", "conv.hip")]
    with ThreadPoolExecutor(4) as ex:
        results = dict(zip(srcs, ex.map(A.audit_source, srcs)))
    bad = {os.path.basename(s): r for s, r in results.items() if r}
    assert not bad, bad


@needs_hipcc
def test_layernorm_backward_prefetch_loop_is_not_drained():
    # the two-row prefetch variants (PF2) of the saved-sum backward, with and without the bias
    # gradient: their row loop must never wait for every outstanding load
    res = A.audit_source(os.path.join(A.CSRC, "layernorm.hip"), drain=r"ln_bwd_kernelILi2ELb0ELb0ELb[01]ELb0ELb1E")
    assert not res, res
