# PMC of the wide global-batch update's row-block form at N = 8 (M = 512):
# where the issue-bound launch spends its cycles.  One counter set per pass.
set -e
T=${1:-r6rb}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/$T/avail.txt 2>&1 || true
N=8 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $R/gpurun_out/$T/p1 -o run --output-format csv -- python3 $R/tools/wgrad_pmc_driver.py > $R/gpurun_out/$T/p1.log 2>&1
N=8 timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $R/gpurun_out/$T/p2 -o run --output-format csv -- python3 $R/tools/wgrad_pmc_driver.py > $R/gpurun_out/$T/p2.log 2>&1
N=8 timeout -s KILL 60 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY -d $R/gpurun_out/$T/p3 -o run --output-format csv -- python3 $R/tools/wgrad_pmc_driver.py > $R/gpurun_out/$T/p3.log 2>&1 || echo "p3 failed"
cd $R
ls gpurun_out/$T/*/
