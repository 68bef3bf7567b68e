set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_skinny.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3p_sk.log 2>&1 || { tail -40 gpurun_out/r3p_sk.log; exit 1; }
tail -1 gpurun_out/r3p_sk.log
for t in 64 128; do WG_TILE=$t timeout -k 10 200 python tools/wide_xact_cost.py > gpurun_out/r3p_cost_$t.json 2> gpurun_out/r3p_cost_$t.err; echo "tile $t: $(cut -c1-120 gpurun_out/r3p_cost_$t.json)"; done
