# Full GPU suite (the driver's round-end form) + smoke + benches + wide kernel stats.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f_suite.log 2>&1 || { tail -60 gpurun_out/r3f_suite.log; exit 1; }
tail -2 gpurun_out/r3f_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f_smoke.log 2>&1 && tail -1 gpurun_out/r3f_smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3f_bench20.json 2> gpurun_out/r3f_bench20.err && cut -c1-220 gpurun_out/r3f_bench20.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 --model 784-128-10 > gpurun_out/r3f_bench_ref.json 2> gpurun_out/r3f_bench_ref.err && cut -c1-220 gpurun_out/r3f_bench_ref.json
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/r3f_stamps2.json 784-128-10 > /dev/null 2>&1 && head -c 600 gpurun_out/r3f_stamps2.json
timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/r3f_wide.json 2> gpurun_out/r3f_wide.err && cut -c1-200 gpurun_out/r3f_wide.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3f_prof -o run -- python $GRAFT_REPO_ROOT/bench_wide.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/r3f_prof.log 2>&1 && cd $GRAFT_REPO_ROOT && python tools/rocpd_summary.py gpurun_out/r3f_prof/run_results.db --skip 200 | cut -c1-160
