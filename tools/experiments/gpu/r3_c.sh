# Round 3: persistent step (restructured) + pk / pk2 data-parallel sums.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c_persist.log 2>&1 || { tail -60 gpurun_out/r3c_persist.log; exit 1; }
tail -1 gpurun_out/r3c_persist.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_xchg.py -x -v -k "pk or auto" --timeout 120 --timeout-method thread > gpurun_out/r3c_xchg.log 2>&1 || { tail -60 gpurun_out/r3c_xchg.log; exit 1; }
tail -1 gpurun_out/r3c_xchg.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3c_bench20.json 2> gpurun_out/r3c_bench20.err && cut -c1-200 gpurun_out/r3c_bench20.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/r3c_bench2000.json 2> gpurun_out/r3c_bench2000.err && cut -c1-200 gpurun_out/r3c_bench2000.json
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/r3c_stamps3.json > /dev/null 2>&1 && cat gpurun_out/r3c_stamps3.json
timeout -k 10 240 python -u tools/pk_probe.py --ranks 1,2,4,8 --algo 0 > gpurun_out/r3c_pk_probe.json 2> gpurun_out/r3c_pk_probe.err && cat gpurun_out/r3c_pk_probe.json
timeout -k 10 240 python -u tools/pk_probe.py --ranks 2,4,8 --algo 1 > gpurun_out/r3c_pk2_probe.json 2> gpurun_out/r3c_pk2_probe.err && cat gpurun_out/r3c_pk2_probe.json
timeout -k 10 300 python -m hipdsml.bench.train_rpc --backend hip --out gpurun_out/r3c_rpc_device_n1.json > /dev/null 2> gpurun_out/r3c_rpc.err && cat gpurun_out/r3c_rpc_device_n1.json
