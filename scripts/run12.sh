set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -x -q -m gpu -k "attention or bert_layer" > gpurun_out/pytest_attn.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/attention_bench.py > gpurun_out/attn_bench.log 2>&1 || exit $?
tail -2 gpurun_out/attn_bench.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_bert_default.log 2>&1 || exit $?
tail -1 gpurun_out/bench_bert_default.log | cut -c1-250
