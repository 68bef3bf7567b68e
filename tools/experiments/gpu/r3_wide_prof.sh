# Wide engine (784-4096-4096-10 bf16) baseline for round 3: bench, head phases, kernel stats.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/r3w_bench.json 2> gpurun_out/r3w_bench.err && cat gpurun_out/r3w_bench.json
timeout -k 10 120 python tools/experiments/head_bench.py > gpurun_out/r3w_head.json 2> gpurun_out/r3w_head.err && cat gpurun_out/r3w_head.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3w_prof -o run -- python $GRAFT_REPO_ROOT/bench_wide.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/r3w_prof.log 2>&1 && cd $GRAFT_REPO_ROOT && find gpurun_out/r3w_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cut -d, -f1-5 {} | head -12
