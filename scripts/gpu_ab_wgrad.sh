#!/bin/bash
# TN wgrad kernel tests + BERT-large step A/B: wgrad kernel (hip/blas) x fused FFN epilogues
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/ab_wgrad"; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py "tests/test_ops2_gpu.py::test_gemm_tn_weight_gradient" "tests/test_ops_gpu.py::test_bert_layer_blocks_match_composed" ${EXTRA_TESTS:-} > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for r in 1 2; do
  for cfg in ${CFGS:-hip:11 blas:11 hip:00}; do
    k=${cfg%%:*}; fd=${cfg##*:}; f=${fd:0:1}; d=${fd:1:1}
    CLOUDTIK_AMD_WGRAD_KERNEL=$k CLOUDTIK_AMD_FUSED_FFN_FWD=$f CLOUDTIK_AMD_FUSED_FFN_DGRAD=$d timeout -k 10 300 python3 "$R/bench.py" --model bert-large --steps 20 --warmup 5 > "$OUT/${k}_${fd}_$r.log" 2>&1 || { echo "run $cfg/$r failed"; tail -5 "$OUT/${k}_${fd}_$r.log"; exit 1; }
    echo "wgrad=$k fused=$fd round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/${k}_${fd}_$r.log") $(grep -o '"loss_last_step": [0-9.]*' "$OUT/${k}_${fd}_$r.log")"
  done
done
