#!/bin/bash
# gemm_nt: numerics tests, then the probe (default staging = LDS-DMA)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py "tests/test_ops_gpu.py::test_bert_layer_blocks_match_composed" > gpurun_out/gemm_stage_tests.log 2>&1 || { tail -30 gpurun_out/gemm_stage_tests.log; exit 1; }
tail -3 gpurun_out/gemm_stage_tests.log
for st in ${STAGES:-0}; do
  PYTHONPATH=. CLOUDTIK_AMD_GEMM_STAGE=$st timeout -k 10 240 python -u bench/gemm_nt_probe.py > gpurun_out/gemm_stage_$st.log 2>&1 || { tail -20 gpurun_out/gemm_stage_$st.log; exit 1; }
  echo "== stage $st"; grep -v amdgpu.ids gpurun_out/gemm_stage_$st.log
done
