#!/bin/bash
# Per-call kernel list of ONE steady ResNet-50 step (name, queue, grid, LDS, us) from a rocprofv3
# kernel trace: which layer each conv / BatchNorm call is, by its grid.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/rn_calls"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/t" -o t -- python3 -u "$R/bench.py" --model resnet50 --steps 4 --warmup 2 > "$OUT/run.log" 2>&1 || { tail -5 "$OUT/run.log"; exit 1; }
tr=$(find "$OUT/t" -name "*kernel_trace.csv" | head -1)
python3 - "$tr" > "$OUT/calls.txt" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
cuts = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
a, b = cuts[-2], cuts[-1]
t0 = int(rows[a]["End_Timestamp"])
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
    print(f'{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{r.get("Queue_Id", r.get("Stream_Id", "?")):>3} '
          f'g{g:>9} lds{r.get("LDS_Block_Size", r.get("Lds_Size", "?")):>6} {r["Kernel_Name"][:90]}')
PY
rm -rf "$OUT/t"
wc -l "$OUT/calls.txt"
