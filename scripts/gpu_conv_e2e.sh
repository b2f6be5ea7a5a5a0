#!/bin/bash
# conv kernel GPU tests, then ResNet-50 bench with the implicit-GEMM convs on / off (same box),
# then a steady-state kernel profile of the on-arm.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/conv_e2e"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_conv_igemm.py tests/test_miopen_solvers.py -m gpu -x -v --timeout 120 \
  --timeout-method thread > "$OUT/tests.txt" 2>&1 || { tail -40 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
for arm in 1 0 1; do
  CLOUDTIK_AMD_CONV_IGEMM=$arm timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 \
    > "$OUT/bench_igemm$arm.log" 2>&1 || { tail -20 "$OUT/bench_igemm$arm.log"; exit 1; }
  echo "igemm=$arm: $(tail -1 "$OUT/bench_igemm$arm.log" | cut -c1-400)"
  grep "kernel audit" "$OUT/bench_igemm$arm.log" | cut -c1-300
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o rn -- python3 -u "$R/bench.py" \
  --model resnet50 --steps 8 --warmup 4 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/prof" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim sgd_kernel --steps 5 --title resnet50_igemm > "$OUT/steady.md"
rm -rf "$OUT/prof"
head -40 "$OUT/steady.md"
