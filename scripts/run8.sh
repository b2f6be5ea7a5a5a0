set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_bert_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bert_default.log | cut -c1-300
bash scripts/gpu_prof.sh bert_mp76 --steps 5 --warmup 2 || exit $?
timeout -k 10 600 python bench.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/bench_rn50.log 2>&1 || exit $?
tail -1 gpurun_out/bench_rn50.log | cut -c1-300
