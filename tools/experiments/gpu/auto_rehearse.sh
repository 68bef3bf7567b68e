# sync=auto end to end on ONE GPU (gloo group; the non-exchange candidate is a
# torch.distributed all-reduce): self-tests, timing of every candidate, choice.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 3; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2964$n bench.py --gpus $n --steps 2000 --warmup 200 --sync auto --rehearse-one-gpu > gpurun_out/rehearse${n}_auto.json 2> gpurun_out/rehearse${n}_auto.err
  grep -v Gloo gpurun_out/rehearse${n}_auto.json
done
