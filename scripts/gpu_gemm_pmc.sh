#!/bin/bash
# Counter passes over the weight-gradient GEMM kernel (one shape): L2 hit/miss, HBM fetch,
# LDS bank conflicts and SQ busy.  Each pass is its own run (counter-block limits).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/gemm_pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
M=${1:-4096}; N=${2:-1024}; S=${3:-4}
i=0
for ctr in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex gemm_tn --output-format csv -d "$OUT/p$i" -o p$i -- python3 "$R/bench/gemm_tn_probe.py" --only $M $N $S > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k}: n={len(v)} mean={sum(v)/len(v):.4g}")
PY
  rm -rf "$OUT/p$i"
done
