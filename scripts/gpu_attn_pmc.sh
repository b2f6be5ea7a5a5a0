#!/bin/bash
# Counter passes over the attention kernels inside the BERT-large bench (a few steps).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/attn_pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export CLOUDTIK_AMD_WGRAD_STREAM=0
RE=${1:-attn_}
i=0
for ctr in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-include-regex "$RE" --output-format csv -d "$OUT/p$i" -o p$i -- python3 "$R/bench.py" --steps 2 --warmup 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in d.items()))
PY
  rm -rf "$OUT/p$i"
done
