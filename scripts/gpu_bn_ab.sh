#!/bin/bash
# BN apply-kernel vectors-per-thread A/B: tests, bench rounds per CLOUDTIK_AMD_BN_EW value, then a
# steady-state kernel profile per value.  scripts/gpu_bn_ab.sh TAG "1 4"
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-bnew}; VALS=${2:-"1 2 4"}
OUT="$R/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$R"
export PYTHONPATH="$R"
for v in $VALS; do
  CLOUDTIK_AMD_BN_EW=$v timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k batchnorm --timeout 120 --timeout-method thread > "$OUT/tests_$v.txt" 2>&1 || { tail -30 "$OUT/tests_$v.txt"; exit 1; }
  echo "EW=$v tests: $(tail -1 "$OUT/tests_$v.txt")"
done
bash "$R/scripts/gpu_ab_env.sh" "$TAG" CLOUDTIK_AMD_BN_EW "$VALS" 2 resnet50 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in $VALS; do
  export CLOUDTIK_AMD_BN_EW=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr$v" -o rn -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4 > "$OUT/prof_$v.log" 2>&1 || { tail -20 "$OUT/prof_$v.log"; exit 1; }
  tr=$(find "$OUT/tr$v" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/steady_profile.py" "$tr" --delim sgd_kernel --steps 5 --title "steady resnet50 BN_EW=$v" > "$OUT/steady_ew$v.md" || exit 1
  rm -rf "$OUT/tr$v"
  grep -E "Steady|bn_" "$OUT/steady_ew$v.md" | cut -c1-150
done
echo ALLDONE
