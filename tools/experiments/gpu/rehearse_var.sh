# 2-rank one-GPU rehearsal variants (timed-step anomaly hunt).
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --gpus 2 --rehearse-one-gpu --no-sync-sweep"
timeout -k 10 200 $B --steps 20 --warmup 5 > gpurun_out/rv_20.json 2> gpurun_out/rv_20.err && tail -1 gpurun_out/rv_20.json
timeout -k 10 200 $B --steps 1000 --warmup 100 --sync xgmi > gpurun_out/rv_xgmi.json 2> gpurun_out/rv_xgmi.err && tail -1 gpurun_out/rv_xgmi.json
timeout -k 10 200 $B --steps 1000 --warmup 100 --sync xgmi --graph-steps 0 > gpurun_out/rv_xgmi_eager.json 2> gpurun_out/rv_xgmi_eager.err && tail -1 gpurun_out/rv_xgmi_eager.json
timeout -k 10 200 $B --steps 100 --warmup 100 --sync xgmi > gpurun_out/rv_xgmi100.json 2> gpurun_out/rv_xgmi100.err && tail -1 gpurun_out/rv_xgmi100.json
