#!/bin/bash
# One GPU session: GPU test suite, both halves of the headline bench, steady-state profiles.
# Usage: scripts/gpu_baseline.sh TAG   (outputs under gpurun_out/TAG/)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-base}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1 || { tail -30 "$OUT/gpu_tests.txt"; exit 1; }
tail -2 "$OUT/gpu_tests.txt"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | cut -c1-600
timeout -k 10 900 python -u bench.py --steps 10 --warmup 3 --compare-eager > "$OUT/bench_eager.log" 2>&1 || { tail -20 "$OUT/bench_eager.log"; exit 1; }
tail -1 "$OUT/bench_eager.log" | cut -c1-900
cd /tmp && export TMPDIR=/tmp
for m in bert-large:lamb_stage1 resnet50:sgd_kernel; do
  name=${m%%:*}; delim=${m##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_$name" -o "$name" -- python3 -u "$R/bench.py" --model $name --steps 8 --warmup 4 > "$OUT/prof_$name.log" 2>&1 || { tail -20 "$OUT/prof_$name.log"; exit 1; }
  tr=$(find "$OUT/tr_$name" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/steady_profile.py" "$tr" --delim "$delim" --steps 5 --title "steady $name" > "$OUT/steady_$name.md" || exit 1
  rm -rf "$OUT/tr_$name"
  head -3 "$OUT/steady_$name.md"
done
echo ALLDONE
