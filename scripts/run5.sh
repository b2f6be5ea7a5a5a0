set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
for b in 64 256; do
timeout -k 10 600 python bench.py --model bert-large --batch $b --steps 10 --warmup 3 --tunableop off > gpurun_out/bench_bert_b$b.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bert_b$b.log | cut -c1-200
done
timeout -k 10 900 python bench.py --model bert-large --batch 256 --steps 3 --warmup 2 --tunableop tune > gpurun_out/tune_bert.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --model resnet50 --batch 256 --steps 3 --warmup 2 --tunableop tune > gpurun_out/tune_rn50.log 2>&1 || exit $?
mkdir -p gpurun_out/tunableop && cp cloudtik_amd/ops/tunableop/* gpurun_out/tunableop/ || true
timeout -k 10 600 python bench.py --model bert-large --batch 256 --steps 10 --warmup 3 --tunableop use > gpurun_out/bench_bert_tuned.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bert_tuned.log | cut -c1-200
timeout -k 10 600 python bench.py --model resnet50 --batch 256 --steps 10 --warmup 3 --tunableop use > gpurun_out/bench_rn50_tuned.log 2>&1 || exit $?
tail -1 gpurun_out/bench_rn50_tuned.log | cut -c1-200
bash scripts/gpu_prof.sh bert256 --model bert-large --batch 256 --steps 5 --warmup 2 --tunableop use || exit $?
