#!/bin/bash
# Counter passes over one conv shape's plain vs BatchNorm-epilogue kernels (bench/conv_epi_one.py)
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/epipmc"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SHAPE=${SHAPE:-64,256,56,1,1}
ARGS="--shape $SHAPE ${EXTRA:-}"
timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex conv_ --output-format csv -d "$OUT/tr" -o tr -- python3 "$R/bench/conv_epi_one.py" $ARGS > "$OUT/tr.log" 2>&1 || { tail -5 "$OUT/tr.log"; exit 1; }
i=0
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VALU_MFMA_MOPS_BF16" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex conv_ --output-format csv -d "$OUT/p$i" -o p$i -- python3 "$R/bench/conv_epi_one.py" $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
tr=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
p=$(find "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 "$OUT"/p4 -name "*counter_collection.csv")
python3 "$R/scripts/pmc_summary.py" --trace "$tr" --pmc $p --raw --title "conv $SHAPE epilogue counters" > "$OUT/pmc.md" || exit 1
rm -rf "$OUT/tr" "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 "$OUT"/p4
cat "$OUT/pmc.md"
