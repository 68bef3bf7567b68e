set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_skinny.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h_tests.log 2>&1 || { tail -30 gpurun_out/r3h_tests.log; exit 1; }
tail -1 gpurun_out/r3h_tests.log
for h in 1 0; do for t in 64 128; do HILO=$h WG_TILE=$t timeout -k 10 200 python tools/wide_xact_cost.py > gpurun_out/r3c_${h}_${t}.json 2> gpurun_out/r3c.err; echo "hilo $h tile $t: $(cut -c1-110 gpurun_out/r3c_${h}_${t}.json)"; done; done
timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/r3h_wide.json 2> gpurun_out/r3h_wide.err && cut -c1-160 gpurun_out/r3h_wide.json
