#!/bin/bash
# BERT-large A/B of the GEMM site routing (ops/transformer.py): hipBLASLt everywhere vs the
# data-gradient sites on the streamed / one-tile MFMA kernels, interleaved, two rounds.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/gemmsites"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest "tests/test_ops_gpu.py::test_bert_layer_blocks_match_composed" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.txt" 2>&1
rc=$?
tail -2 "$O/tests.txt"
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in off "S:do,dx_attn,dx_ffn" "O:do,dx_attn,dx_ffn" "S:do" "O:dx_attn,dx_ffn"; do
    case "$v" in
      off) s=""; o="";;
      S:*) s="${v#S:}"; o="";;
      O:*) s=""; o="${v#O:}";;
    esac
    tag=$(echo "$v" | tr ':,' '__')
    CLOUDTIK_AMD_STREAM_GEMM="$s" CLOUDTIK_AMD_ONETILE_GEMM="$o" timeout -k 10 240 python -u bench.py --model bert-large \
      --steps 20 --warmup 5 > "$O/bert_${tag}_$r.json" 2> "$O/bert_${tag}_$r.err" || exit $?
    echo "$v round $r: $(grep -o '"ms_per_step": [0-9.]*' "$O/bert_${tag}_$r.json")"
  done
done
