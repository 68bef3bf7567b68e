# Hardware counters of the wide-MLP GEMM kernels, one rocprofv3 --pmc pass per
# counter set and kernel (kernel-trace only, no other trace domains).
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for k in rows64 splitk4 dwsgd; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAIT_ANY TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc1_$k -o run --output-format csv -- python3 $R/tools/gemm_one.py $k > $R/gpurun_out/pmc1_$k.log 2>&1
  timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc2_$k -o run --output-format csv -- python3 $R/tools/gemm_one.py $k > $R/gpurun_out/pmc2_$k.log 2>&1
done
ls -R $R/gpurun_out/pmc1_rows64 | head
