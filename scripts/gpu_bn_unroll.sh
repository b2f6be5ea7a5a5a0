#!/bin/bash
# BN reduction rows-in-flight A/B (CLOUDTIK_AMD_BN_UNROLL 4 / 8) x block count, with tests and profiles.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-bnu}"; mkdir -p "$OUT"
cd "$R"; export PYTHONPATH="$R"
for u in 4 8; do
  CLOUDTIK_AMD_BN_UNROLL=$u timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "batchnorm or stem" --timeout 120 --timeout-method thread > "$OUT/tests_$u.txt" 2>&1 || { tail -30 "$OUT/tests_$u.txt"; exit 1; }
  echo "unroll $u tests: $(tail -1 "$OUT/tests_$u.txt")"
done
bash "$R/scripts/gpu_ab_env.sh" "$(basename "$OUT")" CLOUDTIK_AMD_BN_UNROLL "4 8" 2 resnet50 || exit 1
export CLOUDTIK_AMD_BN_UNROLL=8
CLOUDTIK_AMD_BN_BLOCKS=1024 timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > "$OUT/u8_b1024.log" 2>&1 && echo "unroll 8 blocks 1024: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/u8_b1024.log" | head -1)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o rn -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim sgd_kernel --steps 5 --title "steady resnet50 BN unroll 8" > "$OUT/steady_u8.md" || exit 1
rm -rf "$OUT/tr"
grep -E "Steady|bn_stats|bn_bwd_reduce|finalize" "$OUT/steady_u8.md" | cut -c1-150
echo ALLDONE
