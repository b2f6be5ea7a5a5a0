#!/bin/bash
# Two gloo ranks sharing the one GPU, both models in one process with the per-model weight-
# gradient routing (BERT in line, ResNet-50 on the side stream): the configuration that showed
# 1.4 / 1.7 s ResNet steps once (r5c).  Repeats it, then prints per-step ResNet times.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${1:-gloo_mixed}"
mkdir -p "$O"
cd "$R"
rc=0
for i in 1 2 3; do
  env CLOUDTIK_AMD_STEP_PHASES=${PHASES:-0} ${EXTRA_ENV:-} timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --model all --steps 6 --warmup 2 --batch 64 --rn-batch 64 \
      > "$O/mixed_$i.log" 2> "$O/mixed_$i.err" || { rc=$?; echo "run $i failed rc=$rc"; tail -5 "$O/mixed_$i.err"; break; }
  python3 - "$O/mixed_$i.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")]
d = json.loads(l[-1])
print(sys.argv[1].rsplit("/", 1)[1], "bert", d.get("step_ms"), "resnet", d.get("resnet50_step_ms"), "rn host", d.get("resnet50_host_ms"))
PY
done
exit $rc
