# Phase stamps of a 20-step launch: steps 0-7 (the launch's ramp) vs 8-15.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_persist.py -x -q --timeout 120 --timeout-method thread -k "matches_fp32 or launch_split" > gpurun_out/sw_tests.log 2>&1 || { tail -30 gpurun_out/sw_tests.log; exit 1; }
tail -1 gpurun_out/sw_tests.log
for f in 0 8 12; do STAMP_FIRST=$f timeout -k 10 120 python tools/pk_stamps.py gpurun_out/stampwin_$f.json > /dev/null 2>&1; python -c "import json; d=json.load(open('gpurun_out/stampwin_$f.json')); print('first=$f step', d['step_us'], d['layer1'], d['chain'])"; done
