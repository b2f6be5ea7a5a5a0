#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for sk in 1 2 4 8; do
  CLOUDTIK_AMD_WGRAD_STREAM=1 CLOUDTIK_AMD_WGRAD_SPLITK=$sk timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_ws_sk$sk.log 2>&1 || exit 1
  echo "sk=$sk $(tail -1 gpurun_out/bench_ws_sk$sk.log | cut -c1-140)"
done
CLOUDTIK_AMD_WGRAD_STREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_ws0b.log 2>&1 && echo "base $(tail -1 gpurun_out/bench_ws0b.log | cut -c1-140)"
