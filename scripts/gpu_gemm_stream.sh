#!/bin/bash
# Streamed persistent GEMM: correctness tests, then vs one-tile kernel vs hipBLASLt (BERT-large shapes).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/gemmstream"
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gemm_nt_gpu.py "tests/test_ops_gpu.py::test_bert_layer_blocks_match_composed" -m gpu -x -q --timeout 120 --timeout-method thread > "$O/tests.txt" 2>&1
rc=$?
tail -3 "$O/tests.txt"
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" "$O/tests.txt" | head -20; exit $rc; }
timeout -k 10 300 python -u bench/gemm_stream_probe.py --rounds 5 --iters 20 > "$O/probe.jsonl" 2> "$O/probe.md"
rc=$?
tail -12 "$O/probe.md"
[ $rc -eq 0 ] || exit $rc
# BERT-large A/B: hipBLASLt forward / dgrad GEMMs vs every site on the streamed kernel (two rounds)
for r in 1 2; do
  for v in "" all; do
    CLOUDTIK_AMD_STREAM_GEMM=$v timeout -k 10 240 python -u bench.py --model bert-large --steps 20 --warmup 5 \
      > "$O/bert_stream_${v:-off}_$r.json" 2> "$O/bert_stream_${v:-off}_$r.err" || exit $?
    echo "stream=${v:-off} round $r: $(grep -o '"ms_per_step": [0-9.]*' "$O/bert_stream_${v:-off}_$r.json")"
  done
done
