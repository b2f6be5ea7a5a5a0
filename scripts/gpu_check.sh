#!/bin/bash
# One GPU validation pass: op numerics tests, smoke, short bench.  Stops at the first
# crash-like exit (fault/abort/segfault/timeout); plain test failures (rc=1) continue.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
echo "== device"; python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)"
echo "== pytest -m gpu"
timeout -k 10 ${T_TEST:-900} python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; ok $rc || exit $rc
echo "== smoke"
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?
tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for m in ${BENCH_MODELS:-bert-large}; do
  echo "== bench $m"
  timeout -k 10 ${T_BENCH:-600} python bench.py --model $m --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCH_ARGS:-} > gpurun_out/bench_$m.log 2>&1; rc=$?
  tail -3 gpurun_out/bench_$m.log; [ $rc -eq 0 ] || exit $rc
done
