#!/bin/bash
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/attn_check"; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or bert_layer" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 120 python3 "$R/bench/attn_kernel_probe.py" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python3 "$R/bench/attn_kernel_probe.py" --S 512 --B 32 2>&1 | grep -v amdgpu.ids || exit 1
[ "${BENCH:-1}" = 1 ] || exit 0
timeout -k 10 300 python3 "$R/bench.py" --model bert-large --steps 20 --warmup 5 > "$OUT/bert.log" 2>&1 || { tail -5 "$OUT/bert.log"; exit 1; }
echo "bert-large: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bert.log" | head -1)"
