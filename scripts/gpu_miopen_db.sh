#!/bin/bash
# Build a MIOpen user find-db / perf-db for the ResNet-50 training shapes (solver search),
# then re-run the benchmark in immediate mode against that db.
set -o pipefail
mkdir -p gpurun_out/miopen_db
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/gpurun_out/miopen_cache
timeout -k 10 600 python -u bench.py --model resnet50 --conv-benchmark --steps 10 --warmup 3 > gpurun_out/rn50_search.log 2>&1 \
 && tail -1 gpurun_out/rn50_search.log | cut -c1-160 && ls -la gpurun_out/miopen_db \
 && timeout -k 10 300 python -u bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/rn50_db.log 2>&1 \
 && tail -1 gpurun_out/rn50_db.log | cut -c1-160
rm -rf gpurun_out/miopen_cache
