# Wide-MLP tests, step time and per-kernel stats (rocprofv3 kernel trace).
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_gemm_skinny.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wide_pytest.log 2>&1 || { tail -30 gpurun_out/wide_pytest.log; exit 1; }
tail -1 gpurun_out/wide_pytest.log
timeout -k 10 200 python bench_wide.py > gpurun_out/bench_wide.json && cat gpurun_out/bench_wide.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wide -o run -- python3 $R/bench_wide.py --steps 50 --warmup 5 > $R/gpurun_out/prof_wide.log 2>&1
cd $R && find gpurun_out/prof_wide -name "*.db" | head -1 | xargs -I{} python tools/rocpd_summary.py {} --csv gpurun_out/prof_wide_kernels.csv | head -14
