# Data-parallel persistent step (sync=pk) on one GPU: 2/3-process IPC tests, a 2-rank
# rehearsal of bench.py with sync=pk, and the in-kernel phase stamps of rank 0.
# (A granule form of the replica exchange -- {value, step} slots polled directly -- was
# tried: it timed out with 3 processes sharing the GPU; removed.)
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_xchg.py -m gpu -x -q --timeout 150 --timeout-method thread -k "pk" > gpurun_out/pytest_pk.log 2>&1 || { tail -30 gpurun_out/pytest_pk.log; exit 1; }
echo "pk tests: $(tail -1 gpurun_out/pytest_pk.log)"
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --sync pk --steps 1000 --warmup 100 --no-sync-sweep > gpurun_out/pk2.json 2> gpurun_out/pk2.err
grep "^{" gpurun_out/pk2.json | tail -1
timeout -k 10 200 python tools/pk_dp_stamps.py gpurun_out/pk_dp_stamps.json > gpurun_out/pk_dp_stamps.log 2>&1 && cat gpurun_out/pk_dp_stamps.json
