#!/bin/bash
# Detection family on the GPU: tests, inference + training throughput, one rocprof summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_detection.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/det_tests.log 2>&1 \
 && tail -3 gpurun_out/det_tests.log \
 && timeout -k 10 420 python -u examples/ai/inference_benchmark.py > gpurun_out/det_infer.log 2>&1 \
 && cat gpurun_out/det_infer.log | grep '^{' \
 && timeout -k 10 300 python -u examples/ai/inference_benchmark.py --train --models maskrcnn,ssd_resnet34_300 > gpurun_out/det_train.log 2>&1 \
 && grep '^{' gpurun_out/det_train.log \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_maskrcnn -o trace --output-format csv -- python3 examples/ai/inference_benchmark.py --models maskrcnn --steps 5 --warmup 2 > gpurun_out/prof_maskrcnn.log 2>&1 \
 && echo PROF_OK
