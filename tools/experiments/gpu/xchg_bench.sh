# 2-rank rehearsal of bench.py on ONE GPU (gloo group, fused xGMI exchange)
set -e
mkdir -p gpurun_out
python -c "import hipdsml._build as b; b.build()" > gpurun_out/build.log 2>&1
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2000 --warmup 200 --sync xgmi --rehearse-one-gpu > gpurun_out/bench_rehearse2_xgmi.json 2> gpurun_out/bench_rehearse2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --steps 2000 --warmup 200 --sync xgmi --graph-steps 0 --rehearse-one-gpu > gpurun_out/bench_rehearse2_xgmi_eager.json 2>> gpurun_out/bench_rehearse2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 300 --warmup 20 --sync torch --graph-steps 0 --rehearse-one-gpu > gpurun_out/bench_rehearse2_torch.json 2>> gpurun_out/bench_rehearse2.err
cat gpurun_out/bench_rehearse2_*.json
