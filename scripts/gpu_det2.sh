#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_detection.py tests/test_ops2_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/det_tests.log 2>&1 \
 && tail -3 gpurun_out/det_tests.log \
 && timeout -k 10 300 python -u examples/ai/inference_benchmark.py --models maskrcnn,retinanet,yolov4 > gpurun_out/det_infer.log 2>&1 \
 && grep '^{' gpurun_out/det_infer.log \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_maskrcnn_train -o trace --output-format csv -- python3 examples/ai/inference_benchmark.py --train --models maskrcnn --steps 4 --warmup 2 > gpurun_out/prof_maskrcnn_train.log 2>&1 \
 && grep '^{' gpurun_out/prof_maskrcnn_train.log
