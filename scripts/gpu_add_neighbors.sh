#!/bin/bash
# Who launches the remaining elementwise adds in the ResNet-50 step: kernel-trace neighbours.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-addn}"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH="$R"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o rn -- python3 -u "$R/bench.py" --model resnet50 --steps 3 --warmup 2 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/trace_neighbors.py" "$tr" CUDAFunctor_add > "$OUT/add_neighbors.txt"
python3 - "$tr" > "$OUT/add_sizes.txt" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = [i for i, r in enumerate(rows) if "sgd_kernel" in r["Kernel_Name"]]
lo, hi = last[-2], last[-1]
c = collections.Counter()
for r in rows[lo:hi]:
    if "CUDAFunctor_add" in r["Kernel_Name"]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        c[(r.get("Grid_Size", r.get("Grid_Size_X", "?")), round(d))] += 1
for (g, d), n in sorted(c.items(), key=lambda kv: -kv[0][1] * kv[1]):
    print(f"grid {g:>10} ~{d:>5} us x {n}")
PY
rm -rf "$OUT/tr"
cat "$OUT/add_neighbors.txt"; head -30 "$OUT/add_sizes.txt"
echo ALLDONE
