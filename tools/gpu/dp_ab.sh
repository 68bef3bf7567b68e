# Persistent step change A/B: persist + exchange tests, N = 1 stamps and bench,
# lone-replica probes of the Gram DP forms, 2-rank rehearsals.
set -e
T=${1:-dpab}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/${T}_stamps.json > /dev/null 2>&1
python -c "import json; d=json.load(open('gpurun_out/${T}_stamps.json')); print('n1 stamps step', d['step_us'])"
timeout -k 10 100 python bench.py --steps 2000 --warmup 200 2>/dev/null | cut -c1-130
for al in 2 4; do timeout -k 10 200 python tools/pk_probe.py --algo $al --steps 2000 > gpurun_out/${T}_probe_$al.jsonl 2>/dev/null; done
cat gpurun_out/${T}_probe_*.jsonl | cut -c1-100
for m in pkx pkg; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29742 bench.py --gpus 2 --steps 2000 --warmup 200 --sync $m --rehearse-one-gpu > gpurun_out/${T}_reh2_$m.json 2>/dev/null
  grep -v Gloo gpurun_out/${T}_reh2_$m.json | cut -c1-140 || true
done
