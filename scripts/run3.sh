set -u
cd $GRAFT_REPO_ROOT
T_TEST=900 BENCH_MODELS="bert-large resnet50" bash scripts/gpu_check.sh || exit $?
for b in 256; do
  timeout -k 10 600 python bench.py --model bert-large --batch $b --steps 10 --warmup 3 > gpurun_out/bench_bert_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_bert_b$b.log
done
bash scripts/gpu_prof.sh bert256 --model bert-large --batch 256 --steps 5 --warmup 2 || exit $?
bash scripts/gpu_prof.sh rn50 --model resnet50 --batch 256 --steps 5 --warmup 2 || exit $?
