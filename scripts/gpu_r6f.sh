#!/bin/bash
# r6: paired-tile GEMM -- DMA placement variants (CLOUDTIK_AMD_PP_DMA 0/1/2 and the no-DMA timing
# diagnostic 3), numerics checked for 1 and 2.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6f"; mkdir -p "$O"
cd "$R"
for dp in 0 4 3; do  # 1, 2 (DMA in the MFMA slot) measured slower, removed
  chk=""; [ $dp -eq 0 ] || chk="--skip-check"
  CLOUDTIK_AMD_PP_DMA=$dp timeout -k 10 180 python -u bench/gemm_pp_probe.py $chk --rounds 5 --iters 10 \
    --eslots 8 --shapes ffn1_plain,ffn2,ffn1 > "$O/probe_dp$dp.jsonl" 2> "$O/probe_dp$dp.err"
  rc=$?
  cut -c1-600 "$O/probe_dp$dp.jsonl"
  [ $rc -eq 0 ] || { tail -20 "$O/probe_dp$dp.err"; exit $rc; }
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pp_gpu.py \
  > "$O/pytest.log" 2>&1
rc=$?; tail -5 "$O/pytest.log"; exit $rc
