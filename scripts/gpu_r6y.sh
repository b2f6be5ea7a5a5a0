#!/bin/bash
# Counter passes over the LayerNorm kernels (bench/ln_from_y_probe.py): wave anatomy + VALU
# issue, then HBM bytes.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
RE=ln_ CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
  bash scripts/gpu_pmc_cmd.sh bench/ln_from_y_probe.py --rounds 1 --iters 2 && \
RE=ln_ CTRS="FETCH_SIZE" bash scripts/gpu_pmc_cmd.sh bench/ln_from_y_probe.py --rounds 1 --iters 2 && \
RE=ln_ CTRS="WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" bash scripts/gpu_pmc_cmd.sh bench/ln_from_y_probe.py --rounds 1 --iters 2
