# gpu_sim topology with N GPU device servers (CommInit backend "pg"): the GPU
# test and the train_rpc bench at 2 device servers on one GPU.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_pg_bootstrap.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pg_tests.log 2>&1 || { tail -40 gpurun_out/pg_tests.log; exit 1; }
tail -1 gpurun_out/pg_tests.log
timeout -k 10 400 python -m hipdsml.bench.train_rpc --devices 2 --steps 50,937 --reps 5 --out gpurun_out/r4_bench_rpc_device_n2.json > /dev/null 2> gpurun_out/pg_bench.err
cut -c1-900 gpurun_out/r4_bench_rpc_device_n2.json
