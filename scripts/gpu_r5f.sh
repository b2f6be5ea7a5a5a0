#!/bin/bash
# r5: steady-state BERT-large kernel profile at HEAD + forward-site GEMM routing A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r5f}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o bert -- python3 -u "$R/bench.py" --model bert-large --steps 8 --warmup 4 > "$O/prof.log" 2>&1 \
 && tr=$(find "$O/prof" -name "*kernel_trace.csv" | head -1) \
 && python3 "$R/scripts/steady_profile.py" "$tr" --delim lamb_stage1 --steps 5 --top 45 --title "bert-large r5 HEAD" > "$O/steady_bert.md" \
 && rm -rf "$O/prof" && head -12 "$O/steady_bert.md" \
 && cd "$R" && bash "$R/scripts/gpu_ab_cfgs.sh" "$TAG/ab" 2 bert-large "base:" \
      "qkv:CLOUDTIK_AMD_ONETILE_GEMM=qkv,do,dx_attn,dx_ffn" \
      "fwd3:CLOUDTIK_AMD_ONETILE_GEMM=qkv,wo,ffn2,do,dx_attn,dx_ffn"
