# Final tree verification: the driver's round-end steps (GPU suite, smoke,
# bench in driver form) plus the 2,000-step bench and the 784-128-10 model.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=${1:-r4v}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_suite.log 2>&1 || { tail -60 gpurun_out/${T}_suite.log; exit 1; }
tail -2 gpurun_out/${T}_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && tail -1 gpurun_out/${T}_smoke.log
for k in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench20_$k.json 2>/dev/null; cut -c1-150 gpurun_out/${T}_bench20_$k.json; done
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/${T}_bench2000.json 2>/dev/null && cut -c1-150 gpurun_out/${T}_bench2000.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 --model 784-128-10 > gpurun_out/${T}_bench2000_784_128_10.json 2>/dev/null && cut -c1-150 gpurun_out/${T}_bench2000_784_128_10.json
# the N > 1 bench path end to end: 2 ranks sharing the one GPU (gloo group)
timeout -k 10 400 python bench.py --gpus 2 --rehearse-one-gpu --steps 2000 --warmup 200 > gpurun_out/${T}_bench2000_reh2.json 2> gpurun_out/${T}_bench2000_reh2.err && cut -c1-200 gpurun_out/${T}_bench2000_reh2.json
