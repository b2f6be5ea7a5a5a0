#!/bin/bash
# The mixed-policy gloo stall under a HIP API trace: which host calls block.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/gloo_trace"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-trace --output-format csv -d "$OUT/t" -o t -- python3 -u "$R/bench.py" --gpus 2 --dist-backend gloo --model all --steps 6 --warmup 2 --batch 64 --rn-batch 64 > "$OUT/run.log" 2> "$OUT/run.err" || { tail -5 "$OUT/run.err"; exit 1; }
python3 - "$OUT/run.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")]
d = json.loads(l[-1]); print("resnet", d.get("resnet50_step_ms"))
PY
for f in $(find "$OUT/t" -name "*hip_api_trace.csv"); do echo "== $f"; python3 "$R/scripts/api_hotspots.py" "$f" 15; done > "$OUT/hotspots.md"
rm -rf "$OUT/t"
cat "$OUT/hotspots.md" | head -80
