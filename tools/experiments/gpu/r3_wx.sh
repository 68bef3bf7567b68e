set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_skinny.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3x_sk.log 2>&1 || { tail -40 gpurun_out/r3x_sk.log; exit 1; }
tail -1 gpurun_out/r3x_sk.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1 || { tail -40 gpurun_out/r3x_tests.log; exit 1; }
tail -1 gpurun_out/r3x_tests.log
timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/r3x_wide.json 2> gpurun_out/r3x_wide.err && cut -c1-160 gpurun_out/r3x_wide.json
timeout -k 10 200 python tools/wide_xact_cost.py > gpurun_out/r3x_cost.json 2> gpurun_out/r3x_cost.err && cat gpurun_out/r3x_cost.json
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 120 python tools/experiments/head_bench.py > gpurun_out/r3h_head.json 2> gpurun_out/r3h_head.err && cat gpurun_out/r3h_head.json
