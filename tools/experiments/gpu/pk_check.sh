# Persistent-step check: its tests, smoke, and the N=1 bench (persistent vs three-launch).
set -e
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_persist.py -x -v --timeout 60 --timeout-method thread > gpurun_out/pytest_pk.log 2>&1 || { tail -40 gpurun_out/pytest_pk.log; exit 1; }
tail -3 gpurun_out/pytest_pk.log
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 100 python bench.py --steps 20 --warmup 5 2>/dev/null
timeout -k 10 100 python bench.py 2>/dev/null
HIPDSML_PERSIST=0 timeout -k 10 100 python bench.py 2>/dev/null
