set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_deform_gpu.py tests/test_data_gpu.py -x -q -m gpu > gpurun_out/pytest_new_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_new_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python examples/ai/spark_parquet_resnet50.py --data-path /tmp/ct_pq --epochs 3 > gpurun_out/pipeline_rn50.log 2>&1 || exit $?
tail -1 gpurun_out/pipeline_rn50.log
timeout -k 10 600 python bench/gbdt_bench.py > gpurun_out/gbdt_bench.log 2>&1 || exit $?
tail -1 gpurun_out/gbdt_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_gbdt -o gbdt -- python $GRAFT_REPO_ROOT/bench/gbdt_bench.py --rounds 20 > $GRAFT_REPO_ROOT/gpurun_out/gbdt_prof.log 2>&1 || exit $?
echo done
