# Persistent-step launch overhead after batching the prologue loads: persistent GPU tests,
# launch overhead breakdown, driver-form bench x3.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1 || { tail -30 gpurun_out/pytest_sub.log; exit 1; }
tail -1 gpurun_out/pytest_sub.log
timeout -k 10 240 python -u tools/pk_overhead.py gpurun_out/pk_overhead.json > gpurun_out/pk_overhead.log 2>&1 && python -c "import json;d=json.load(open('gpurun_out/pk_overhead.json'));print(d['persistent'], d['n20_kernel_edges_us'], d['empty_launch_sync_us'])"
for r in 1 2 3; do timeout -k 10 120 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys;print('driver form', json.load(sys.stdin)['ms_per_step'])"; done
