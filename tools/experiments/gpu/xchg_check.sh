set -e
mkdir -p gpurun_out
python -c "import hipdsml._build as b; b.build()" > gpurun_out/build.log 2>&1
timeout -k 10 300 python -m pytest tests/test_gpu_xchg.py -m gpu -x -q > gpurun_out/pytest_xchg.log 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
tail -3 gpurun_out/pytest_xchg.log gpurun_out/pytest_gpu.log
