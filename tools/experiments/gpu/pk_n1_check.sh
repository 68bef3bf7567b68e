# N=1 persistent step after templating out the replica exchange, plus the pk tests / rehearsal.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -m gpu -x -q --timeout 150 --timeout-method thread -k "persist or pk" > gpurun_out/pytest_pk.log 2>&1 || { tail -30 gpurun_out/pytest_pk.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/pytest_pk.log)"
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys;print('driver form', json.load(sys.stdin)['ms_per_step'])"
  timeout -k 10 120 python bench.py 2>/dev/null | python -c "import json,sys;print('2000 steps', json.load(sys.stdin)['ms_per_step'])"
done
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 1000 --warmup 100 > gpurun_out/auto2.json 2> gpurun_out/auto2.err
grep "^{" gpurun_out/auto2.json | tail -1
