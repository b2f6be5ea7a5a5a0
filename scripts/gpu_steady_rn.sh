#!/bin/bash
# ResNet-50 steady-state kernel profile (WS=0: gradient side stream off)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/steady"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
name=resnet50${TAG:-}
CLOUDTIK_AMD_WGRAD_STREAM=${WS:-1} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o $name -- python3 -u "$R/bench.py" --model resnet50 --steps 8 --warmup 4 > "$OUT/$name.log" 2>&1 || exit $?
tr=$(find "$OUT/$name" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim sgd_kernel --steps 5 --top 40 --gaps ${GAPS:-0} --title "$name" > "$OUT/$name.md" || exit $?
rm -rf "$OUT/$name"
head -26 "$OUT/$name.md"
