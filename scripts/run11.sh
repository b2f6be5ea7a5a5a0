set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/ops_bench.py > gpurun_out/ops_bench.log 2>&1 || exit $?
tail -1 gpurun_out/ops_bench.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_bert_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bert_default.log | cut -c1-250
