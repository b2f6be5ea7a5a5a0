#!/bin/bash
# Round GPU check: GPU test suite, smoke, short benches. Each step has its own time limit;
# steps are chained so the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
 && tail -3 gpurun_out/gpu_tests.log \
 && timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2>&1 \
 && tail -1 gpurun_out/bench_bert.log \
 && timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_rn50.log 2>&1 \
 && tail -1 gpurun_out/bench_rn50.log
