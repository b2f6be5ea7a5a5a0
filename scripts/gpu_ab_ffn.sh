#!/bin/bash
# BERT-large step A/B of the fused FFN GEMM epilogues: FWD DGRAD in {00, 10, 01, 11}, 2 rounds
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/ab_ffn"; mkdir -p "$OUT"
for r in 1 2; do
  for fd in ${COMBOS:-00 10 01 11}; do
    f=${fd:0:1}; d=${fd:1:1}
    CLOUDTIK_AMD_FUSED_FFN_FWD=$f CLOUDTIK_AMD_FUSED_FFN_DGRAD=$d timeout -k 10 300 python3 "$R/bench.py" --model bert-large --steps 20 --warmup 5 > "$OUT/ffn_${fd}_$r.log" 2>&1 || { echo "run $fd/$r failed"; tail -5 "$OUT/ffn_${fd}_$r.log"; exit 1; }
    echo "fwd=$f dgrad=$d round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/ffn_${fd}_$r.log") $(grep -o '"step_ms_ci95": [0-9.]*' "$OUT/ffn_${fd}_$r.log")"
  done
done
