#!/bin/bash
# One counter pass (SQ wave anatomy + LDS) over the kernels matching $RE of a python command.
#   RE=ln_bwd bash scripts/gpu_pmc_cmd.sh bench/ops_bench.py [args]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_cmd"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}
script="$1"; shift
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-include-regex "${RE:-.}" --output-format csv -d "$OUT/p" -o p -- python3 "$R/$script" "$@" > "$OUT/p.log" 2>&1 || { echo "pmc failed"; tail -5 "$OUT/p.log"; exit 1; }
f=$(find "$OUT/p" -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in d.items()))
PY
rm -rf "$OUT/p"
