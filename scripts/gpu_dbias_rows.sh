#!/bin/bash
# GEMM / transformer GPU tests, the epilogue probe and a BERT A/B of the spread bias-gradient atomics.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/dbias_rows"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py tests/test_ops_gpu.py tests/test_model_parity.py -k "gemm or ffn or bert or transformer or block or lamb or sumsq or optim or embedding" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 120 python3 bench/epi_burst_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
bash "$R/scripts/gpu_ab_cfgs.sh" dbias_rows/ab 2 bert-large "base:" "rows1:CLOUDTIK_AMD_DBIAS_ROWS=1"
