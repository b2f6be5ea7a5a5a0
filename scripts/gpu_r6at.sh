#!/bin/bash
# SSD-ResNet34 training: stem knobs A/B, then kernel stats with the in-tree conv path on / off.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6at"; mkdir -p "$O"
cd "$R"
for v in "CLOUDTIK_AMD_NOOP=1" "CLOUDTIK_AMD_STEM_FOLD=0" "CLOUDTIK_AMD_STEM_PAIRS=0" "CLOUDTIK_AMD_CONV_IGEMM=0"; do
  env $v timeout -k 10 300 python -u examples/ai/inference_benchmark.py --models ssd_resnet34_300 --train > "$O/s.log" 2>&1 || { echo "$v failed"; tail -5 "$O/s.log"; exit 1; }
  echo "$v: $(grep '^{' "$O/s.log" | tail -1 | grep -o '"ms_per_batch": [0-9.]*')"
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  env CLOUDTIK_AMD_CONV_IGEMM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/p$v" -o ssd -- python3 -u "$R/examples/ai/inference_benchmark.py" --models ssd_resnet34_300 --train > "$O/p$v.log" 2>&1 || { tail -5 "$O/p$v.log"; exit 1; }
  f=$(find "$O/p$v" -name "*kernel_stats.csv" | head -1)
  echo "== igemm=$v"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):5d}  {r["Name"][:100]}')
PY
  rm -rf "$O/p$v"
done
