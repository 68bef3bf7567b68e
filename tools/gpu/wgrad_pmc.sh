# PMC counters of the wide global-batch update (M = 512) at tile 64 and 128.
set -e
T=${1:-wp}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/wide_xact_cost.py > gpurun_out/${T}_xact64.json 2>/dev/null && cat gpurun_out/${T}_xact64.json
WG_TILE=128 timeout -k 10 200 python tools/wide_xact_cost.py > gpurun_out/${T}_xact128.json 2>/dev/null && cat gpurun_out/${T}_xact128.json
cd /tmp && export TMPDIR=/tmp
for tl in 64 128; do
  WG_TILE=$tl timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_p1_$tl -o run --output-format csv -- python3 $R/tools/wgrad_pmc_driver.py > $R/gpurun_out/${T}_p1_$tl.log 2>&1
  WG_TILE=$tl timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_p2_$tl -o run --output-format csv -- python3 $R/tools/wgrad_pmc_driver.py > $R/gpurun_out/${T}_p2_$tl.log 2>&1
done
cd $R
python tools/pmc_summary.py gpurun_out/${T}_pmc.json t64=wgrad_multi_k:gpurun_out/${T}_p1_64,gpurun_out/${T}_p2_64 t128=wgrad_multi_big_k:gpurun_out/${T}_p1_128,gpurun_out/${T}_p2_128 > /dev/null
cat gpurun_out/${T}_pmc.json
