#!/bin/bash
# r6: the data-parallel path after moving the collectives to their own comm stream: the GPU
# bucketer tests, then two gloo ranks sharing the GPU with both models in one process (the
# r5 "mixed routing" stall configuration, gloo_stall.md), bucket waits > 50 ms printed.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/${TAG:-r6c}"; mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_ddp_gloo.py tests/test_bucket_ready_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/ddp_gpu.txt" 2>&1 || { tail -30 "$O/ddp_gpu.txt"; exit 1; }
tail -1 "$O/ddp_gpu.txt"
rc=0
for i in 1 2; do
  env CLOUDTIK_AMD_STEP_PHASES=50 timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --model all --steps 6 --warmup 2 --batch 64 --rn-batch 64 --baseline-steps 0 \
      > "$O/mixed_$i.log" 2> "$O/mixed_$i.err" || { rc=$?; echo "run $i failed rc=$rc"; tail -5 "$O/mixed_$i.err"; break; }
  python3 - "$O/mixed_$i.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")]
d = json.loads(l[-1])
print(sys.argv[1].rsplit("/", 1)[1], "bert", d.get("step_ms"), "resnet", d.get("resnet50_step_ms"))
print("  grad", d["config"]["grad_dtype"], "rn buckets", [(b["bucket"], b.get("done_ms_vs_backward_end"), b.get("host_wait_ms")) for b in (d.get("resnet50_bucket_timeline") or [])])
PY
  grep -c "bucket waits" "$O/mixed_$i.err" || true
done
exit $rc
