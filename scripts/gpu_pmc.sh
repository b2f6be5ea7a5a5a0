#!/bin/bash
# Hardware-counter passes over the hot kernels of one bench model (each pass its own run,
# within the per-block counter limits), plus a kernel-trace run for durations.
# Usage: scripts/gpu_pmc.sh TAG MODEL [kernel-regex]
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; MODEL=$2; RE=${3:-.}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export CLOUDTIK_AMD_WGRAD_STREAM=0 CLOUDTIK_BENCH_AUDIT=0
ARGS="--model $MODEL --steps 2 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "$RE" --output-format csv -d "$OUT/tr" -o tr -- python3 "$R/bench.py" $ARGS > "$OUT/tr.log" 2>&1 || { tail -5 "$OUT/tr.log"; exit 1; }
i=0
for ctr in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-include-regex "$RE" --output-format csv -d "$OUT/p$i" -o p$i -- python3 "$R/bench.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
tr=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
p=$(find "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 -name "*counter_collection.csv")
python3 "$R/scripts/pmc_summary.py" --trace "$tr" --pmc $p --title "$MODEL counters" > "$OUT/pmc_$MODEL.md" || exit 1
rm -rf "$OUT/tr" "$OUT/p1" "$OUT/p2" "$OUT/p3"
head -30 "$OUT/pmc_$MODEL.md"
