# Row-block global-batch update: tests, then the xact cost at N = 1/2/4/8 with
# the 16x16x32 and 32x32x16 MFMA forms alternating, then PMC of both at N = 8.
# Record of the A/B in profiles/r6_wide_xact_cost.json: it ran on commit
# 34d37d2; the 32x32x16 form (HIPDSML_RB_MFMA32) was removed after it measured
# no faster, so on later trees both arms run the 16x16x32 kernel.
set -e
T=${1:-r6rbab}
R=$GRAFT_REPO_ROOT
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_skinny.py -k "rowblk or wgrad" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for m in 0 1; do
    HIPDSML_RB_MFMA32=$m timeout -k 10 200 python tools/wide_xact_cost.py > $O/cost_${m}_$k.json 2>/dev/null
    echo "m32=$m $(cut -c1-160 $O/cost_${m}_$k.json)"
  done
done
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  HIPDSML_RB_MFMA32=$m N=8 timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $R/$O/p1_$m -o run --output-format csv -- python3 $R/tools/wgrad_pmc_driver.py > $R/$O/p1_$m.log 2>&1
  HIPDSML_RB_MFMA32=$m N=8 timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $R/$O/p2_$m -o run --output-format csv -- python3 $R/tools/wgrad_pmc_driver.py > $R/$O/p2_$m.log 2>&1
done
