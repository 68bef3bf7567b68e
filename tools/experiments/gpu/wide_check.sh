set -e
mkdir -p gpurun_out
python -c "import hipdsml._build as b; b.build()" > gpurun_out/build.log 2>&1
timeout -k 10 300 python -m pytest tests/test_gpu_wide.py tests/test_gpu_dp.py tests/test_gpu_fit.py -m gpu -x -q > gpurun_out/pytest_wide.log 2>&1
timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/gemm_bench.json
timeout -k 10 300 python bench_wide.py > gpurun_out/bench_wide.json 2> gpurun_out/bench_wide.err
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wide -o run -- python3 $R/bench_wide.py --steps 50 --warmup 5 > $R/gpurun_out/prof_wide.log 2>&1
cat $R/gpurun_out/bench_wide.json $R/gpurun_out/gemm_bench.json
tail -n 3 $R/gpurun_out/pytest_wide.log
