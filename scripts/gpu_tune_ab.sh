#!/bin/bash
# BERT-large with the in-tree TunableOp table vs TunableOp off vs the table without the forward
# projection entries (qkv / wo / ffn2), interleaved on one box.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out/tune_ab"
P="$R/gpurun_out/tune_ab/pruned.csv"
grep -v -e "tn_3072_32768_1024_ld_1024_1024_3072" -e "tn_1024_32768_1024_ld_1024_1024_1024" \
        -e "tn_1024_32768_4096_ld_4096_4096_1024" "$R/cloudtik_amd/ops/tunableop/gfx950_tunableop.csv" > "$P"
wc -l "$P"
bash "$R/scripts/gpu_ab_cfgs.sh" tune_ab/ab 2 bert-large "base:" "off:CLOUDTIK_BENCH_TUNABLEOP=off" "pruned:CLOUDTIK_BENCH_TUNE_FILE=$P"
