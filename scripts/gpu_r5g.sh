#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r5g}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
timeout -k 10 120 python -u bench/epi_burst_probe.py > "$O/epi.txt" 2>&1 && cat "$O/epi.txt" \
 && CLOUDTIK_AMD_GEMM_DIAG=4 timeout -k 10 120 python -u bench/epi_burst_probe.py > "$O/epi_diag4.txt" 2>&1 && cat "$O/epi_diag4.txt" \
 && timeout -k 10 200 python -u bench/audit_probe.py > "$O/audit.txt" 2>&1 && tail -1 "$O/audit.txt" \
 && bash "$R/scripts/gpu_ab_cfgs.sh" "$TAG/ab" 2 bert-large "base:" \
      "qkv:CLOUDTIK_AMD_ONETILE_GEMM=qkv,do,dx_attn,dx_ffn" \
      "fwd3:CLOUDTIK_AMD_ONETILE_GEMM=qkv,wo,ffn2,do,dx_attn,dx_ffn"
