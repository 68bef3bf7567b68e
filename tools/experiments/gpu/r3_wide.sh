# Wide engine: tests, bench, per-kernel stats.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_gemm_skinny.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w_tests.log 2>&1 || { tail -60 gpurun_out/r3w_tests.log; exit 1; }
tail -1 gpurun_out/r3w_tests.log
timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/r3w_bench.json 2> gpurun_out/r3w_bench.err && cat gpurun_out/r3w_bench.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3w_prof -o run -- python $GRAFT_REPO_ROOT/bench_wide.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/r3w_prof.log 2>&1 && cd $GRAFT_REPO_ROOT && python tools/rocpd_summary.py gpurun_out/r3w_prof/run_results.db --skip 200 | cut -c1-160
