# Single-replica persistent step after a kernel change: its tests, phase
# stamps, and the bench in driver form (20 steps) and over 2,000 steps.
# Usage: bash tools/gpu/pk_n1_ab.sh TAG
set -e
T=${1:-n1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_persist.log 2>&1 || { tail -40 gpurun_out/${T}_persist.log; exit 1; }
tail -1 gpurun_out/${T}_persist.log
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/${T}_stamps.json > /dev/null 2> gpurun_out/${T}_stamps.err
python -c "import json; d=json.load(open('gpurun_out/${T}_stamps.json')); print('stamps step', d['step_us'], d.get('gram'))"
for k in 1 2 3; do timeout -k 10 100 python bench.py --steps 20 --warmup 5 2>/dev/null | cut -c1-150; done
timeout -k 10 100 python bench.py --steps 2000 --warmup 200 2>/dev/null | cut -c1-150
