set -e
for al in 4 2; do timeout -k 10 200 python tools/pk_probe.py --algo $al --steps 2000 --stamps gpurun_out/hp2_probe_stamps_$al.jsonl > gpurun_out/hp2_probe_$al.jsonl 2> gpurun_out/hp2_probe_$al.err; cat gpurun_out/hp2_probe_$al.jsonl; done
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29742 bench.py --gpus 2 --steps 2000 --warmup 200 --sync pkx --rehearse-one-gpu --no-sync-sweep --no-allreduce-probe 2>/dev/null | grep -v Gloo | cut -c1-200
