set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $R/gpurun_out/pmc/attn1 -o attn -- python3 $R/bench/attention_bench.py > $R/gpurun_out/pmc/attn1.log 2>&1; echo rc1=$?
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc/attn2 -o attn -- python3 $R/bench/attention_bench.py > $R/gpurun_out/pmc/attn2.log 2>&1; echo rc2=$?
ls -R $R/gpurun_out/pmc | head -30
