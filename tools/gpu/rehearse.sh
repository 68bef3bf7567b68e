# N-rank plumbing of bench.py on ONE GPU (gloo stands in for RCCL; "rehearsal": true).
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 3; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2974$n bench.py --gpus $n --steps 2000 --warmup 200 --sync auto --rehearse-one-gpu > gpurun_out/reh${n}.json 2> gpurun_out/reh${n}.err
  grep -v Gloo gpurun_out/reh${n}.json | cut -c1-900
done
