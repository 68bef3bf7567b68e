# Round-end style check on one GPU: every GPU test, smoke(), the headline bench,
# and 2-rank rehearsals of bench.py (replicas share cuda:0, gloo group).
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
for s in xact xgmi; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2963${#s} bench.py --gpus 2 --steps 2000 --warmup 200 --sync $s --rehearse-one-gpu > gpurun_out/rehearse2_$s.json 2> gpurun_out/rehearse2_$s.err
  cat gpurun_out/rehearse2_$s.json
done
