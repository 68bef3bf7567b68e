# Round 3: restructured persistent step (56 layer-1 + 4 chains + 4 gradient
# blocks, 2- and 3-layer models, batch <= 64): tests, smoke, N=1 bench (driver
# form and 2000 steps), phase stamps of both models, pk 2/3-process tests.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3b_persist.log 2>&1 || { tail -60 gpurun_out/r3b_persist.log; exit 1; }
tail -1 gpurun_out/r3b_persist.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b_smoke.log 2>&1 && tail -1 gpurun_out/r3b_smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b_bench20.json 2> gpurun_out/r3b_bench20.err && cat gpurun_out/r3b_bench20.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r3b_bench2000.json 2> gpurun_out/r3b_bench2000.err && cat gpurun_out/r3b_bench2000.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 --model 784-128-10 > gpurun_out/r3b_bench2000_ref.json 2> gpurun_out/r3b_bench2000_ref.err && cat gpurun_out/r3b_bench2000_ref.json
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/r3b_stamps3.json > /dev/null 2>&1 && cat gpurun_out/r3b_stamps3.json
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/r3b_stamps2.json 784-128-10 > /dev/null 2>&1 && cat gpurun_out/r3b_stamps2.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_xchg.py -x -v -k "pk or auto" --timeout 120 --timeout-method thread > gpurun_out/r3b_xchg.log 2>&1 || { tail -60 gpurun_out/r3b_xchg.log; exit 1; }
tail -1 gpurun_out/r3b_xchg.log
timeout -k 10 300 python -m hipdsml.bench.train_rpc --backend hip --out gpurun_out/r3b_rpc_device_n1.json > /dev/null 2> gpurun_out/r3b_rpc.err && cat gpurun_out/r3b_rpc_device_n1.json
