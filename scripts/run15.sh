set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_graph_gpu.py -x -q -m gpu -k gbdt > gpurun_out/pytest_gbdt_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gbdt_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/gbdt_bench.py > gpurun_out/gbdt_bench.log 2>&1 || exit $?
tail -1 gpurun_out/gbdt_bench.log
timeout -k 10 600 python bench/gbdt_bench.py --rows 10000000 --rounds 50 > gpurun_out/gbdt_bench_10m.log 2>&1 || exit $?
tail -1 gpurun_out/gbdt_bench_10m.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_gbdt2 -o gbdt -- python $GRAFT_REPO_ROOT/bench/gbdt_bench.py --rounds 20 > $GRAFT_REPO_ROOT/gpurun_out/gbdt_prof2.log 2>&1 || exit $?
echo done
