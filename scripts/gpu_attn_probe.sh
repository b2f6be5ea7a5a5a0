#!/bin/bash
# attention kernel times + counter passes (one pass per block group)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/attn_probe"; mkdir -p "$OUT"
timeout -k 10 120 python3 "$R/bench/attn_kernel_probe.py" 2>&1 | grep -v amdgpu.ids || exit 1
[ "${PMC:-1}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
i=0
for ctr in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex attn_ --output-format csv -d "$OUT/p$i" -o p$i -- python3 "$R/bench/attn_kernel_probe.py" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
  f=$(find "$OUT/p$i" -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:34]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, " ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in d.items()))
PY
  rm -rf "$OUT/p$i"
done
