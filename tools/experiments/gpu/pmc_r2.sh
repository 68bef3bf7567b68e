# Round-2 wide GEMM counters: the split-K skinny kernels and the weight-gradient
# kernel next to the round-1 kernels they replace (one --pmc pass per counter set).
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for k in rows64 skinny_nt skinny_nn dwsgd wgrad; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TA_TA_BUSY GRBM_GUI_ACTIVE -d $R/gpurun_out/p1_$k -o run --output-format csv -- python3 $R/tools/gemm_one.py $k > $R/gpurun_out/p1_$k.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/p2_$k -o run --output-format csv -- python3 $R/tools/gemm_one.py $k > $R/gpurun_out/p2_$k.log 2>&1
done
cd $R && python tools/pmc_summary.py gpurun_out/pmc_r2.json rows64=gemm_rows64:gpurun_out/p1_rows64,gpurun_out/p2_rows64 skinny_nt=gemm_skinny_k:gpurun_out/p1_skinny_nt,gpurun_out/p2_skinny_nt skinny_nn=gemm_skinny_k:gpurun_out/p1_skinny_nn,gpurun_out/p2_skinny_nn dwsgd=gemm_bf16_nt_k:gpurun_out/p1_dwsgd,gpurun_out/p2_dwsgd wgrad=wgrad_sgd_k:gpurun_out/p1_wgrad,gpurun_out/p2_wgrad > /dev/null && echo pmc ok
