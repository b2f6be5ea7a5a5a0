#!/bin/bash
# gloo two-rank, two-model rehearsal (the r5 "mixed routing" stall) at more hardware queues per
# process: does the stall track queue sharing?  GPU_MAX_HW_QUEUES 4 (box default) vs 16.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6ak"; mkdir -p "$O"
cd "$R"
for q in 16 4; do
  env GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --model all --steps 6 --warmup 2 \
      --batch 64 --rn-batch 64 --baseline-steps 0 > "$O/q$q.log" 2> "$O/q$q.err" || { echo "q=$q failed"; tail -5 "$O/q$q.err"; exit 1; }
  python3 - "$O/q$q.log" "$q" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print("queues", sys.argv[2], "bert", d.get("step_ms"), "resnet", d.get("resnet50_step_ms"))
PY
done
