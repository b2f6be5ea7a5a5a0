#!/bin/bash
# DLRM step time on the final tree: default vs weight gradients in line vs hipBLASLt weight
# gradients, then a kernel-time summary of the default.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/r6an"; mkdir -p "$O"
cd "$R"
for v in "CLOUDTIK_AMD_NOOP=1" "CLOUDTIK_AMD_WGRAD_STREAM=0" "CLOUDTIK_AMD_WGRAD_KERNEL=blas" "CLOUDTIK_AMD_NOOP=2"; do
  env $v timeout -k 10 200 python -u examples/ai/dlrm_synthetic.py --steps 60 > "$O/run.log" 2>&1 || { tail -5 "$O/run.log"; exit 1; }
  echo "$v: $(grep '^{' "$O/run.log" | tail -1 | cut -c1-140)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o dlrm -- python3 -u "$R/examples/ai/dlrm_synthetic.py" --steps 60 > "$O/prof.log" 2>&1 || { tail -5 "$O/prof.log"; exit 1; }
f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"kernel time total {tot/1e6:.1f} ms over 65 steps -> {tot/1e6/65:.3f} ms/step")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6/65:8.4f} ms/step {int(r["Calls"])//65:4d}/step  {r["Name"][:90]}')
PY
rm -rf "$O/prof"
