# Persistent step: tests (single replica + pk/pk2 exchanges), phase stamps of
# both models, driver-form and 2000-step benches.  Usage: bash tools/gpu/pk_check.sh TAG
set -e
T=${1:-pk}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/${T}_stamps3.json > /dev/null 2>&1
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/${T}_stamps2.json 784-128-10 > /dev/null 2>&1
python -c "
import json,sys
for f in sys.argv[1:]:
    d=json.load(open(f)); print(f, json.dumps({k:d[k] for k in d if k!='model'}))" gpurun_out/${T}_stamps3.json gpurun_out/${T}_stamps2.json
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench20.json 2> gpurun_out/${T}_bench20.err && cut -c1-200 gpurun_out/${T}_bench20.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/${T}_bench2000.json 2> gpurun_out/${T}_bench2000.err && cut -c1-200 gpurun_out/${T}_bench2000.json
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 --model 784-128-10 > gpurun_out/${T}_bench_ref.json 2> gpurun_out/${T}_bench_ref.err && cut -c1-200 gpurun_out/${T}_bench_ref.json
