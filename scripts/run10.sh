set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python examples/ai/mnist_mlp.py --epochs 2 > gpurun_out/mnist_gpu.log 2>&1 || exit $?
tail -1 gpurun_out/mnist_gpu.log | cut -c1-250
timeout -k 10 400 python examples/ai/resnet50_synthetic.py --batch-size 256 --num-iters 3 --num-batches-per-iter 5 --num-warmup-batches 3 > gpurun_out/rn50_example.log 2>&1 || exit $?
tail -2 gpurun_out/rn50_example.log
timeout -k 10 400 python examples/ai/resnet50_synthetic.py --horovod --fp16-allreduce --batch-size 256 --num-iters 3 --num-batches-per-iter 5 --num-warmup-batches 3 > gpurun_out/rn50_hvd.log 2>&1 || exit $?
tail -1 gpurun_out/rn50_hvd.log
timeout -k 10 400 python examples/ai/dlrm_synthetic.py --batch-per-rank 2048 --steps 30 > gpurun_out/dlrm_gpu.log 2>&1 || exit $?
tail -1 gpurun_out/dlrm_gpu.log
