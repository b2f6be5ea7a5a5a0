set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench/attention_bench.py > gpurun_out/attn_bench.log 2>&1 || exit $?
tail -1 gpurun_out/attn_bench.log
timeout -k 10 600 python bench.py --model bert-large --batch 256 --steps 10 --warmup 3 > gpurun_out/bench_bert_b256.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bert_b256.log | cut -c1-250
