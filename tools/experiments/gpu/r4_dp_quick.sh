# Data-parallel persistent forms after a kernel change: mirror / IPC tests,
# lone-replica probe (pkx, pkg) with stamps, 2-rank rehearsal.  Usage: bash tools/gpu/dp_quick.sh TAG
set -e
T=${1:-dq}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread -k "persist or mirror or pkx or pkg or many" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for al in 4 2; do timeout -k 10 200 python tools/pk_probe.py --algo $al --steps 2000 --stamps gpurun_out/${T}_probe_stamps_$al.jsonl > gpurun_out/${T}_probe_$al.jsonl 2> gpurun_out/${T}_probe_$al.err; cat gpurun_out/${T}_probe_$al.jsonl; done
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29742 bench.py --gpus 2 --steps 2000 --warmup 200 --sync pkx --rehearse-one-gpu --no-sync-sweep --no-allreduce-probe > gpurun_out/${T}_reh2.json 2>/dev/null
grep -v Gloo gpurun_out/${T}_reh2.json | cut -c1-200
