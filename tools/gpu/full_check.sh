set -e
python -c "import hipdsml._build as b; b.build()" > gpurun_out/build.log 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_fit.py tests/test_gpu_kernels.py tests/test_gpu_wide.py tests/test_gpu_dp.py tests/test_gpu_rpc.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 python bench_wide.py > gpurun_out/bench_wide.json 2> gpurun_out/bench_wide.err
cat gpurun_out/bench.json gpurun_out/bench_wide.json
tail -3 gpurun_out/pytest_gpu.log
