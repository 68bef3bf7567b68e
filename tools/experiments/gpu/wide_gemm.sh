# Wide-MLP GEMM tests + microbenchmarks + the wide step (skinny weight-stream kernel).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wide_pytest.log 2>&1 || { tail -30 gpurun_out/wide_pytest.log; exit 1; }
tail -2 gpurun_out/wide_pytest.log
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gemm_bench.json
timeout -k 10 200 python bench_wide.py > gpurun_out/bench_wide.json
cat gpurun_out/gemm_bench.json gpurun_out/bench_wide.json
