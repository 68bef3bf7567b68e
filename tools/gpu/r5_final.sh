# Final-tree check: the whole GPU suite (one process), smoke(), the driver's
# bench form x3 and a 2,000-step run, the wide bench.
set -e
T=${1:-r5f}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
for k in 1 2 3; do timeout -k 10 300 python bench.py 2>/dev/null; done > gpurun_out/${T}_bench_default.jsonl
cut -c1-160 gpurun_out/${T}_bench_default.jsonl
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --no-e2e 2>/dev/null > gpurun_out/${T}_bench2000.json
cut -c1-160 gpurun_out/${T}_bench2000.json
timeout -k 10 300 python bench_wide.py --steps 200 --warmup 20 2>/dev/null > gpurun_out/${T}_wide.json
cut -c1-160 gpurun_out/${T}_wide.json
