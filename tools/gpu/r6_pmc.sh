# Round-6 PMC records of the final tree: the single-replica persistent step
# (one pass, 2000 steps) and every kernel of the wide step (three passes).
set -e -o pipefail
T=${1:-r6p}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_sr1 -o run --output-format csv -- python3 $R/bench.py --steps 2000 --warmup 200 --no-e2e > $R/gpurun_out/${T}_sr1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_sr2 -o run --output-format csv -- python3 $R/bench.py --steps 2000 --warmup 200 --no-e2e > $R/gpurun_out/${T}_sr2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_sr3 -o run --output-format csv -- python3 $R/bench.py --steps 2000 --warmup 200 --no-e2e > $R/gpurun_out/${T}_sr3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_w1 -o run --output-format csv -- python3 $R/bench_wide.py --steps 30 --warmup 5 > $R/gpurun_out/${T}_w1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_w2 -o run --output-format csv -- python3 $R/bench_wide.py --steps 30 --warmup 5 > $R/gpurun_out/${T}_w2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_MISS_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_w3 -o run --output-format csv -- python3 $R/bench_wide.py --steps 30 --warmup 5 > $R/gpurun_out/${T}_w3.log 2>&1
cd $R
S=gpurun_out/${T}_sr1,gpurun_out/${T}_sr2,gpurun_out/${T}_sr3
python tools/pmc_summary.py gpurun_out/${T}_pmc_persist.json "persist=mlp_persist_k:$S" > /dev/null
D=gpurun_out/${T}_w1,gpurun_out/${T}_w2,gpurun_out/${T}_w3
python tools/pmc_summary.py gpurun_out/${T}_pmc_wide.json "skinny_nt=gemm_skinny_k<false>:$D" "skinny_nn=gemm_skinny_k<true>:$D" "head=head_softmax_xent_k:$D" "update_plus_input=wgrad_multi_in_k:$D" > /dev/null
cat gpurun_out/${T}_pmc_persist.json gpurun_out/${T}_pmc_wide.json
