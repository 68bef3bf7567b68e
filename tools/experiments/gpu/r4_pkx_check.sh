# Exchange-free data-parallel Gram form (pkx): persistent + exchange GPU tests,
# the lone-replica probe of every persistent form at N = 1/2/4/8, then 2-rank
# one-GPU rehearsals of bench.py.  Usage: bash tools/gpu/pkx_check.sh TAG [modes]
set -e
T=${1:-pkx}
MODES=${2:-"pkx pkg"}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread -k "persist or pkx or pkg or auto or many" > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for al in 4 2 0; do
  timeout -k 10 200 python tools/pk_probe.py --algo $al --steps 2000 --stamps gpurun_out/${T}_probe_stamps_$al.jsonl > gpurun_out/${T}_probe_$al.jsonl 2> gpurun_out/${T}_probe_$al.err
  cat gpurun_out/${T}_probe_$al.jsonl
done
for m in $MODES; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29742 bench.py --gpus 2 --steps 2000 --warmup 200 --sync $m --rehearse-one-gpu --no-sync-sweep --no-allreduce-probe > gpurun_out/${T}_reh2_$m.json 2> gpurun_out/${T}_reh2_$m.err
  grep -v Gloo gpurun_out/${T}_reh2_$m.json | cut -c1-400
done
