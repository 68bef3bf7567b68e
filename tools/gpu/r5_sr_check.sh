# Single-replica persistent step after a layer-1 change: persistent tests, bench
# (2000 steps and the driver's 20-step form x3), one PMC pass (LDS conflicts).
set -e
T=${1:-sr}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_gram.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --no-e2e > gpurun_out/${T}_b2000.json 2>/dev/null
cut -c1-140 gpurun_out/${T}_b2000.json
for k in 1 2 3; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-e2e 2>/dev/null | cut -c1-140; done > gpurun_out/${T}_b20.json
cat gpurun_out/${T}_b20.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_p1 -o run --output-format csv -- python3 $R/bench.py --steps 2000 --warmup 200 --no-e2e > $R/gpurun_out/${T}_p1.log 2>&1
cd $R
python tools/pmc_summary.py gpurun_out/${T}_pmc.json persist=mlp_persist_k:gpurun_out/${T}_p1 > /dev/null
cat gpurun_out/${T}_pmc.json
