#!/bin/bash
# attention forward 16-byte stores: attention GPU tests, the kernel probe, BERT-large bench twice
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/attnstore"; mkdir -p "$O"; cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "attn or attention or bert" --timeout 120 --timeout-method thread > "$O/tests.txt" 2>&1
rc=$?; tail -2 "$O/tests.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench/attn_kernel_probe.py > "$O/probe.txt" 2>&1 || { tail -5 "$O/probe.txt"; exit 1; }
tail -6 "$O/probe.txt"
for r in 1 2; do
  timeout -k 10 240 python -u bench.py --model bert-large --steps 20 --warmup 5 > "$O/bert_$r.json" 2>/dev/null || exit 1
  grep -o '"ms_per_step": [0-9.]*' "$O/bert_$r.json"
done
