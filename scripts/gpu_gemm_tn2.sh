#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py > gpurun_out/gemm_tn2_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tn2_tests.log; exit 1; }
tail -3 gpurun_out/gemm_tn2_tests.log
timeout -k 10 300 python -u bench/gemm_tn2_probe.py > gpurun_out/gemm_tn2_probe.log 2>&1 || { tail -20 gpurun_out/gemm_tn2_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gemm_tn2_probe.log
