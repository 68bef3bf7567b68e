# Round-4 baseline on the round-3 tree: full GPU suite, smoke, driver-form
# bench, launch fixed cost, rocprofv3 kernel trace and PMC passes of the
# single-replica persistent step (mlp_persist_k<3,0>).
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4s_suite.log 2>&1 || { tail -60 gpurun_out/r4s_suite.log; exit 1; }
tail -2 gpurun_out/r4s_suite.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4s_bench20.json 2> gpurun_out/r4s_bench20.err && cut -c1-200 gpurun_out/r4s_bench20.json
timeout -k 10 300 python tools/pk_overhead.py gpurun_out/r4s_overhead.json > gpurun_out/r4s_overhead.log 2>&1 && tail -c 900 gpurun_out/r4s_overhead.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4s_prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/r4s_prof.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4s_prof2k -o run -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/r4s_prof2k.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $R/gpurun_out/r4s_p1 -o run --output-format csv -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/r4s_p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/r4s_p2 -o run --output-format csv -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/r4s_p2.log 2>&1
cd $R
python tools/pmc_summary.py gpurun_out/r4s_pmc.json persist=mlp_persist_k:gpurun_out/r4s_p1,gpurun_out/r4s_p2 | head -30
for d in r4s_prof r4s_prof2k; do find gpurun_out/$d -name "*.db" | head -1 | xargs -I{} python tools/rocpd_summary.py {} --csv gpurun_out/${d}_kernels.csv | cut -c1-180 | head -12; done
