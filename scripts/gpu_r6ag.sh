#!/bin/bash
# From-output LayerNorm backward: load-then-copy prefetch (3 waves/SIMD) vs two register sets
# (CLOUDTIK_AMD_LN_BWD_PF2_Y=1, 2 waves/SIMD); LN GPU tests with it on, probe + step A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
CLOUDTIK_AMD_LN_BWD_PF2_Y=1 timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py tests/test_model_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6ag_tests.txt 2>&1 || { tail -30 gpurun_out/r6ag_tests.txt; exit 1; }
tail -1 gpurun_out/r6ag_tests.txt
for r in 1 2 3; do
  for v in 0 1; do
    CLOUDTIK_AMD_LN_BWD_PF2_Y=$v timeout -k 10 120 python3 bench/ln_from_y_probe.py --rounds 3 2>/dev/null | tail -1 | sed "s/^/pf2y=$v: /" || exit 1
  done
done
bash "$R/scripts/gpu_ab_env.sh" r6ag_step CLOUDTIK_AMD_LN_BWD_PF2_Y "0 1" 3
