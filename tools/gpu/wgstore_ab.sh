# Update epilogue with the four split-master stores issued together (no
# store-data reuse wait): wgrad / wide tests, then staged old / new builds
# alternating: the wide bench and the update cost.
set -e
T=${1:-ws}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_skinny.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 1 2 3; do
  for v in old new; do
    echo -n "$v wide "; (cd abtmp/$v && timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 2>/dev/null | cut -c1-100)
  done
done
for k in 1 2; do
  for v in old new; do
    echo -n "$v xact "; (cd abtmp/$v && timeout -k 10 200 python tools/wide_xact_cost.py 2>/dev/null | cut -c1-100)
  done
done
