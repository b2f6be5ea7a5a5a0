set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench/gbdt_bench.py > gpurun_out/gbdt_bench.log 2>&1 || exit $?
tail -1 gpurun_out/gbdt_bench.log
timeout -k 10 600 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/rn50_default.log 2>&1 || exit $?
tail -2 gpurun_out/rn50_default.log | cut -c1-300
timeout -k 10 900 python bench.py --model resnet50 --steps 20 --warmup 5 --conv-benchmark > gpurun_out/rn50_find.log 2>&1 || exit $?
tail -2 gpurun_out/rn50_find.log | cut -c1-300
echo done
