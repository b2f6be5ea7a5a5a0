#!/bin/bash
# Counter passes over the HIP gemm_nt kernel vs hipBLASLt on one shape.
# Usage: scripts/gpu_gemm_nt_pmc.sh TAG M N K
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; shift
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH="$R"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o tr -- python3 "$R/bench/gemm_nt_one.py" "$@" > "$OUT/tr.log" 2>&1 || { tail -5 "$OUT/tr.log"; exit 1; }
i=0
for ctr in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/p$i" -o p$i -- python3 "$R/bench/gemm_nt_one.py" "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
done
tr=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
p=$(find "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 "$OUT"/p4 "$OUT"/p5 -name "*counter_collection.csv" 2>/dev/null)
python3 "$R/scripts/pmc_summary.py" --trace "$tr" --pmc $p --title "gemm_nt $* counters" --raw > "$OUT/pmc_gemm_nt.md" || exit 1
cat "$OUT/pmc_gemm_nt.md"
