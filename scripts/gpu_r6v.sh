#!/bin/bash
# LayerNorm backward with two rows in flight per wave (CLOUDTIK_AMD_LN_BWD_PF2): LN GPU tests,
# kernel probe A/B (interleaved), then the BERT-large step A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/r6v"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -m gpu -k layernorm -x -q --timeout 120 --timeout-method thread \
  > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -2 "$OUT/tests.txt"
for r in 1 2 3; do
  for v in 0 1; do
    CLOUDTIK_AMD_LN_BWD_PF2=$v timeout -k 10 120 python3 bench/ln_from_y_probe.py --rounds 3 > "$OUT/probe_${v}_$r.json" 2>&1 \
      || { cat "$OUT/probe_${v}_$r.json"; exit 1; }
    echo "pf2=$v: $(cat "$OUT/probe_${v}_$r.json")"
  done
done
bash "$R/scripts/gpu_ab_env.sh" r6v_step CLOUDTIK_AMD_LN_BWD_PF2 "0 1" 3
