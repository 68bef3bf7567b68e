# Row-block update with cost-balanced runs: tests, xact cost (8 / 4 waves), stamps
# (record of the round-6 A/B: the 8-wave form was removed afterwards, HIPDSML_RB_WAVES is no longer read)
set -e
O=gpurun_out/${1:-r6rbbal}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_skinny.py -k "rowblk or wgrad" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  for wv in 8 4; do
    HIPDSML_RB_WAVES=$wv timeout -k 10 200 python tools/wide_xact_cost.py > $O/cost_${wv}_$k.json 2>/dev/null
    echo "waves=$wv $(cut -c1-130 $O/cost_${wv}_$k.json)"
  done
done
cp tools/measure_so/_C.so distributed-machine-learning-pipeline_amd/_C.so
for wv in 8 4; do HIPDSML_RB_WAVES=$wv timeout -k 10 100 python tools/rowblk_stamps.py > $O/s_$wv.json 2> $O/e_$wv.log; echo "stamps waves=$wv $(cat $O/s_$wv.json)"; done
