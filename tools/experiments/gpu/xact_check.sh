# Activation exchange (xact) on ONE GPU: exchange tests, then 2- and 3-rank
# rehearsals of bench.py (gloo group, replicas sharing cuda:0) for xact vs xgmi.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_xchg.py -x -v --timeout 120 --timeout-method thread > gpurun_out/xact_pytest.log 2>&1
for n in 2 3; do
  for s in xact xgmi; do
    timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2962$n bench.py --gpus $n --steps 2000 --warmup 200 --sync $s --rehearse-one-gpu > gpurun_out/rehearse${n}_$s.json 2> gpurun_out/rehearse${n}_$s.err
  done
done
tail -3 gpurun_out/xact_pytest.log
cat gpurun_out/rehearse*.json
