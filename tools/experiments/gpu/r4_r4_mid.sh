# Mid-round check: full GPU suite, smoke, driver-form bench, RPC all-reduce experiment.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m_suite.log 2>&1 || { tail -60 gpurun_out/r4m_suite.log; exit 1; }
tail -2 gpurun_out/r4m_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4m_smoke.log 2>&1 && tail -1 gpurun_out/r4m_smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4m_bench20.json 2> gpurun_out/r4m_bench20.err && cut -c1-200 gpurun_out/r4m_bench20.json
bash tools/gpu/rpc_ar.sh
