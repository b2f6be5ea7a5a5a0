#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_detection.py tests/test_ops2_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/det_tests.log 2>&1 \
 && tail -2 gpurun_out/det_tests.log \
 && timeout -k 10 300 python -u examples/ai/inference_benchmark.py --train --models maskrcnn,retinanet --steps 5 > gpurun_out/det_train.log 2>&1 \
 && grep '^{' gpurun_out/det_train.log \
 && timeout -k 10 400 python -u examples/ai/inference_benchmark.py --train --conv-benchmark --models maskrcnn,retinanet --steps 5 > gpurun_out/det_train_cb.log 2>&1 \
 && grep '^{' gpurun_out/det_train_cb.log \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_maskrcnn_train -o trace --output-format csv -- python3 examples/ai/inference_benchmark.py --train --models maskrcnn --steps 4 --warmup 2 > gpurun_out/prof_maskrcnn_train.log 2>&1 \
 && grep '^{' gpurun_out/prof_maskrcnn_train.log
