set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_graph_gpu.py -x -q -m gpu -k gbdt > gpurun_out/pytest_gbdt_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gbdt_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/gbdt_bench.py > gpurun_out/gbdt_bench.log 2>&1 || exit $?
tail -1 gpurun_out/gbdt_bench.log
timeout -k 10 600 python bench/gbdt_bench.py --rows 10000000 --rounds 50 > gpurun_out/gbdt_bench_10m.log 2>&1 || exit $?
tail -1 gpurun_out/gbdt_bench_10m.log
timeout -k 10 900 python applications/fraud_detection/train.py > gpurun_out/fraud.log 2>&1 || exit $?
tail -1 gpurun_out/fraud.log
echo done
