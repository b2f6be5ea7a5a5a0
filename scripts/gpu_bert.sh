#!/bin/bash
# BERT kernels: op numerics tests, BERT-large bench, steady-state profile (serial kernels).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-bert}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_model_parity.py tests/test_ops2_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 300 python -u bench.py --model bert-large --steps 20 --warmup 5 > "$OUT/bench_bert.log" 2>&1 || { tail -20 "$OUT/bench_bert.log"; exit 1; }
tail -1 "$OUT/bench_bert.log" | cut -c1-260
cd /tmp && export TMPDIR=/tmp
for ws in 1 0; do
  CLOUDTIK_AMD_WGRAD_STREAM=$ws timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr$ws" -o bert -- python3 -u "$R/bench.py" --model bert-large --steps 8 --warmup 4 > "$OUT/prof$ws.log" 2>&1 || { tail -20 "$OUT/prof$ws.log"; exit 1; }
  tr=$(find "$OUT/tr$ws" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/steady_profile.py" "$tr" --delim lamb_stage1 --steps 5 --title "steady bert-large (wgrad stream $ws)" > "$OUT/steady_bert_ws$ws.md" || exit 1
  rm -rf "$OUT/tr$ws"
done
head -24 "$OUT/steady_bert_ws0.md"
echo ALLDONE
