#!/bin/bash
# conv wgrad on the side stream: GPU tests, ResNet-50 A/B, steady profile.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-conv1x1}"; mkdir -p "$OUT"
cd "$R"; export PYTHONPATH="$R"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q -k "conv or deferred or stem or linear or optimizer" --timeout 120 --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
bash "$R/scripts/gpu_ab_env.sh" "$(basename "$OUT")" CLOUDTIK_AMD_CONV_WGRAD_STREAM "0 1" 2 resnet50 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o rn -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim sgd_kernel --steps 5 --top 40 --title "steady resnet50 conv wgrad side stream" > "$OUT/steady.md" || exit 1
rm -rf "$OUT/tr"
grep -E "Steady|add|Cijk|igemm_bwd|Cast|fill" "$OUT/steady.md" | cut -c1-160
echo ALLDONE
