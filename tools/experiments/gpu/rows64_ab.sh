# Wide step's first-layer GEMM (K = 784): 8-wave single-batch form vs the 4-wave form.
set -e
mkdir -p gpurun_out
HIPDSML_ROWS64_MID=1 timeout -k 10 200 python -m pytest tests/test_gpu_wide.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pt_rows.log 2>&1 || { tail -20 gpurun_out/pt_rows.log; exit 1; }
echo "wide tests: $(tail -1 gpurun_out/pt_rows.log)"
for r in 1 2; do for m in 0 1; do
  HIPDSML_ROWS64_MID=$m timeout -k 10 200 python bench_wide.py > gpurun_out/bw_$m.json 2>/dev/null
  echo "mid8=$m $(python -c "import json;print(json.load(open('gpurun_out/bw_$m.json'))['ms_per_step'])")"
done; done
