set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_graph_gpu.py -x -q -m gpu > gpurun_out/pytest_graph.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_graph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1200 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_all.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_all.log; exit $rc
