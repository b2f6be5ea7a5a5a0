#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench/wgrad_stream_check.py \
 && CLOUDTIK_AMD_WGRAD_STREAM=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_ws0.log 2>&1 \
 && tail -1 gpurun_out/bench_ws0.log | cut -c1-200 \
 && CLOUDTIK_AMD_WGRAD_STREAM=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_ws1.log 2>&1 \
 && tail -1 gpurun_out/bench_ws1.log | cut -c1-200
