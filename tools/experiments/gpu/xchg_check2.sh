set -e
mkdir -p gpurun_out
python -c "import hipdsml._build as b; b.build()" > gpurun_out/build.log 2>&1
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_gpu_xchg.py -m gpu -x -q > gpurun_out/pytest_xchg.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2000 --warmup 200 --sync xgmi --rehearse-one-gpu > gpurun_out/bench_rehearse2_xgmi.json 2> gpurun_out/bench_rehearse2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 3 --steps 2000 --warmup 200 --sync xgmi --rehearse-one-gpu > gpurun_out/bench_rehearse3_xgmi.json 2>> gpurun_out/bench_rehearse2.err
cat gpurun_out/bench_rehearse*_xgmi.json
tail -n 3 gpurun_out/pytest_xchg.log
