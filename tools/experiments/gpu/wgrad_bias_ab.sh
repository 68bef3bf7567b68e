# Wide weight update with the bias column sums spread over 256 threads: tests, launch A/B, step.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -m pytest tests/test_gpu_wide.py tests/test_gpu_dp.py -m gpu -q -x --timeout 150 --timeout-method thread > gpurun_out/pt_wb.log 2>&1 || { tail -20 gpurun_out/pt_wb.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/pt_wb.log)"
timeout -k 10 200 python tools/wgrad_var.py 2>/dev/null | tail -1
for r in 1 2 3; do timeout -k 10 200 python bench_wide.py 2>/dev/null | python -c "import json,sys;print('wide', json.load(sys.stdin)['ms_per_step'])"; done
