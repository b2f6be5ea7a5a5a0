#!/bin/bash
# Fused ResNet stem (BN + ReLU + max-pool): GPU numerics test, ResNet-50 bench x2, steady profile.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-stem}"; mkdir -p "$OUT"
cd "$R"; export PYTHONPATH="$R"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "stem or batchnorm" --timeout 120 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > "$OUT/bench_$r.log" 2>&1 || { tail -20 "$OUT/bench_$r.log"; exit 1; }
  echo "round $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_$r.log" | head -1) $(grep -o '"value": [0-9.]*' "$OUT/bench_$r.log" | head -1)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o rn -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim sgd_kernel --steps 5 --top 40 --title "steady resnet50 fused stem" > "$OUT/steady.md" || exit 1
rm -rf "$OUT/tr"
grep -E "Steady|pool|bn_apply|bn_bwd_apply|fill" "$OUT/steady.md" | cut -c1-160
echo ALLDONE
