# Persistent step: tests, phase stamps, bench.
set -e
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_persist.py -x -q --timeout 60 --timeout-method thread > gpurun_out/pytest_pk.log 2>&1 || { tail -40 gpurun_out/pytest_pk.log; exit 1; }
tail -1 gpurun_out/pytest_pk.log
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/pk_stamps.json 2>&1 | grep -v amdgpu.ids
timeout -k 10 100 python bench.py 2>/dev/null
