#!/bin/bash
# Two gloo ranks sharing the one GPU: ResNet-50 alone, and both models with every weight gradient
# on the side stream / in line, to tell a policy-switch stall from gloo's own behaviour.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-gloo}"
mkdir -p "$O"
cd "$R"
run() { # tag env... -- args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 8 --warmup 2 --batch 64 --rn-batch 64 \
      --model "${MODEL:-all}" > "$O/$tag.log" 2> "$O/$tag.err"
}
MODEL=resnet50 run rn_only CLOUDTIK_X=1 \
 && run all_side CLOUDTIK_AMD_WGRAD_STREAM=1 \
 && run all_inline CLOUDTIK_AMD_WGRAD_STREAM=0 \
 && MODEL=resnet50 run rn_only_inline CLOUDTIK_AMD_WGRAD_STREAM=0
rc=$?
for f in "$O"/*.log; do python - "$f" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")]
if l:
    d = json.loads(l[-1]); k = "resnet50_step_ms" if "resnet50_step_ms" in d else "step_ms"
    print(sys.argv[1].rsplit("/", 1)[1], d.get("metric"), d.get(k), d.get("resnet50_per_rank_step_ms") or d.get("per_rank_step_ms"))
PY
done
exit $rc
