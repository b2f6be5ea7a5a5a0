#!/bin/bash
# BN tests + ResNet-50 bench + a short trace and the neighbours of the fill / add kernels.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/${1:-rnn}"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "batchnorm" > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > "$OUT/bench_rn50.log" 2>&1 || { tail -20 "$OUT/bench_rn50.log"; exit 1; }
tail -1 "$OUT/bench_rn50.log" | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o rn -- python3 -u "$R/bench.py" --model resnet50 --steps 3 --warmup 2 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
tr=$(find "$OUT/tr" -name "*kernel_trace.csv" | head -1)
python3 "$R/scripts/steady_profile.py" "$tr" --delim sgd_kernel --steps 2 --title "steady resnet50" > "$OUT/steady_resnet50.md"
grep -E "finalize|stats|reduce" "$OUT/steady_resnet50.md"
python3 "$R/scripts/trace_neighbors.py" "$tr" SubTensorOp
python3 "$R/scripts/trace_neighbors.py" "$tr" CUDAFunctor_add
python3 "$R/scripts/trace_neighbors.py" "$tr" fillBufferAligned
rm -rf "$OUT/tr"
