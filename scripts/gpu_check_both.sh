#!/bin/bash
# kernel tests touched by the current change, then BERT-large and ResNet-50 benches (defaults)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/check_both"; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_nt_gpu.py tests/test_conv_igemm.py "tests/test_ops2_gpu.py::test_gemm_tn_weight_gradient" "tests/test_ops_gpu.py::test_bert_layer_blocks_match_composed" ${EXTRA_TESTS:-} > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for r in $(seq 1 ${ROUNDS:-1}); do
  for m in ${MODELS:-bert-large resnet50}; do
    timeout -k 10 300 python3 "$R/bench.py" --model $m --steps 20 --warmup 5 > "$OUT/${m}_$r.log" 2>&1 || { echo "bench $m failed"; tail -8 "$OUT/${m}_$r.log"; exit 1; }
    echo "$m round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/${m}_$r.log" | head -1) $(grep -o '"loss_last_step": [0-9.]*' "$OUT/${m}_$r.log" | head -1)"
  done
done
