#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rnnt.py tests/test_more_models.py tests/test_detection.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/models_tests.log 2>&1 \
 && tail -2 gpurun_out/models_tests.log \
 && timeout -k 10 400 python -u examples/ai/inference_benchmark.py --models rnnt,t5_base,transnetv2,maskrcnn --steps 5 --warmup 2 > gpurun_out/models_infer.log 2>&1 \
 && grep '^{' gpurun_out/models_infer.log \
 && timeout -k 10 400 python -u examples/ai/inference_benchmark.py --train --models rnnt,t5_base,maskrcnn --steps 10 --warmup 5 > gpurun_out/models_train.log 2>&1 \
 && grep '^{' gpurun_out/models_train.log
