#!/bin/bash
# LayerNorm backward from the output (CLOUDTIK_AMD_LN_FROM_Y) re-measured after the
# unconditional-load change: BERT-large step A/B, 3 interleaved rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
bash "$R/scripts/gpu_ab_env.sh" r6w_step CLOUDTIK_AMD_LN_FROM_Y "0 1" 3
