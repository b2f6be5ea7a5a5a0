#!/bin/bash
# Attention kernel A/B on the BERT-large shape: persistent vs one-item-per-workgroup grids and
# forward occupancy variants, after the attention GPU tests.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/attn_ab"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn or bert" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
# VARIANTS: comma-separated "persist:wpe" pairs
IFS=, read -r -a VS <<< "${VARIANTS:-1:2,0:2,1:3,0:3}"
for v in "${VS[@]}"; do
  export CLOUDTIK_AMD_ATTN_FWD_PIPE=${PIPE:-1}
  set -- ${v/:/ }
  CLOUDTIK_AMD_ATTN_PERSIST=$1 CLOUDTIK_AMD_ATTN_FWD_WPE=$2 timeout -k 10 120 python3 bench/attn_kernel_probe.py 2>&1 | grep -v amdgpu.ids | sed "s/^/persist=$1 wpe=$2 /" || exit 1
done
CLOUDTIK_AMD_ATTN_PERSIST=1 timeout -k 10 120 python3 bench/attn_kernel_probe.py --S 512 --B 32 2>&1 | grep -v amdgpu.ids | sed "s/^/persist=1 S512 /" || exit 1
CLOUDTIK_AMD_ATTN_PERSIST=0 timeout -k 10 120 python3 bench/attn_kernel_probe.py --S 512 --B 32 2>&1 | grep -v amdgpu.ids | sed "s/^/persist=0 S512 /" || exit 1
[ "${BENCH:-0}" = 1 ] || exit 0
timeout -k 10 300 python3 bench.py --model bert-large --steps 20 --warmup 5 > "$OUT/bert.log" 2>&1 || { tail -5 "$OUT/bert.log"; exit 1; }
echo "bert-large: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bert.log" | head -1)"
