#!/bin/bash
# Attention forward: global_load_lds K/V staging (CLOUDTIK_AMD_ATTN_FWD_GLDS) vs register
# staging, at the forward's occupancy variants, after the attention GPU tests.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/attn_gl"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or attn" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
IFS=, read -r -a VS <<< "${VARIANTS:-0:2,1:3,1:2,1:4}"
for rep in 1 2; do
for v in "${VS[@]}"; do
  set -- ${v/:/ }
  for shape in "--S 128 --B 256 --p 0.1" "--S 128 --B 256 --p 0.0" "--S 512 --B 32 --p 0.1"; do
    CLOUDTIK_AMD_ATTN_FWD_GLDS=$1 CLOUDTIK_AMD_ATTN_FWD_WPE=$2 timeout -k 10 120 python3 bench/attn_kernel_probe.py $shape 2>&1 | grep -v amdgpu.ids | sed "s/^/gl=$1 wpe=$2 /" || exit 1
  done
done
done
[ "${BENCH:-0}" = 1 ] || exit 0
for rep in 1 2; do
for g in 0 1; do
  CLOUDTIK_AMD_ATTN_FWD_GLDS=$g timeout -k 10 300 python3 bench.py --model bert-large --steps 20 --warmup 5 > "$OUT/bert_$g.log" 2>&1 || { tail -5 "$OUT/bert_$g.log"; exit 1; }
  echo "gl=$g bert-large: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bert_$g.log" | head -1)"
done
done
