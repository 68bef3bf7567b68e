# Round 3, first GPU pass: multi-replica tests with the 3-step self-test,
# pk lone-replica probe at N = 1/2/4/8, 2- and 3-rank one-GPU rehearsals of
# bench.py (sync=auto; replicas_identical must be true).
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_xchg.py tests/test_gpu_persist.py tests/test_gpu_dp.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3a_pytest.log 2>&1 || { tail -60 gpurun_out/r3a_pytest.log; exit 1; }
tail -1 gpurun_out/r3a_pytest.log
timeout -k 10 240 python -u tools/pk_probe.py --ranks 1,2,4,8 > gpurun_out/r3a_pk_probe.json 2> gpurun_out/r3a_pk_probe.err
cat gpurun_out/r3a_pk_probe.json
for n in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2964$n bench.py --gpus $n --steps 2000 --warmup 200 --sync auto --rehearse-one-gpu > gpurun_out/r3a_rehearse${n}.json 2> gpurun_out/r3a_rehearse${n}.err
  grep -v Gloo gpurun_out/r3a_rehearse${n}.json
done
