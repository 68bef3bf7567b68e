# Data-parallel Gram form: persistent + exchange GPU tests, then 2-rank one-GPU
# rehearsals of bench.py with each persistent sync mode.  Usage: bash tools/gpu/pkg_check.sh TAG
set -e
T=${1:-pkg}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for m in pkg pk pkg2 auto; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29742 bench.py --gpus 2 --steps 2000 --warmup 200 --sync $m --rehearse-one-gpu > gpurun_out/${T}_reh2_$m.json 2> gpurun_out/${T}_reh2_$m.err
  grep -v Gloo gpurun_out/${T}_reh2_$m.json | cut -c1-700
done
