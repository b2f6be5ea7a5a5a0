#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_detection.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/det_tests.log 2>&1 \
 && tail -1 gpurun_out/det_tests.log \
 && timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_rn50.log 2>&1 \
 && tail -1 gpurun_out/bench_rn50.log \
 && timeout -k 10 300 python -u examples/ai/inference_benchmark.py --train --models maskrcnn,retinanet,ssd_resnet34_300 --steps 5 > gpurun_out/det_train.log 2>&1 \
 && grep '^{' gpurun_out/det_train.log
