# Row-block update with 8-wave workgroups (two waves a SIMD): tests, then the
# xact cost at N = 1/2/4/8 alternating 4 / 8 waves
set -e
O=gpurun_out/${1:-r6rb8}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_skinny.py -k "rowblk or wgrad" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  for wv in 4 8; do
    HIPDSML_RB_WAVES=$wv timeout -k 10 200 python tools/wide_xact_cost.py > $O/cost_${wv}_$k.json 2>/dev/null
    echo "waves=$wv $(cut -c1-130 $O/cost_${wv}_$k.json)"
  done
done
