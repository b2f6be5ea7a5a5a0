#!/bin/bash
# Detection GPU check: tests, Mask R-CNN train/inference throughput, kernel stats of training.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_detection.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/det_tests.log 2>&1 \
 && tail -1 gpurun_out/det_tests.log \
 && timeout -k 10 300 python -u examples/ai/inference_benchmark.py --train --models maskrcnn --steps 10 --warmup 5 > gpurun_out/det_train.log 2>&1 \
 && grep '^{' gpurun_out/det_train.log \
 && timeout -k 10 300 python -u examples/ai/inference_benchmark.py --models maskrcnn,fasterrcnn,retinanet --steps 10 --warmup 5 > gpurun_out/det_infer.log 2>&1 \
 && grep '^{' gpurun_out/det_infer.log \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_det -o det --output-format csv -- python3 -u examples/ai/inference_benchmark.py --train --models maskrcnn --steps 5 --warmup 3 > gpurun_out/det_prof.log 2>&1 \
 && echo prof-ok
