# Row-block run balancing: the segment-overhead constant of the cost model, swept
set -e
O=gpurun_out/${1:-r6ov2}
mkdir -p $O
for k in 1 2 3; do
  for ov in 1.0 1.5 2.0 2.3; do
    HIPDSML_RB_OV=$ov timeout -k 10 200 python tools/wide_xact_cost.py > $O/c_${ov}_$k.json 2>/dev/null
    echo "ov=$ov $(cut -c1-110 $O/c_${ov}_$k.json)"
  done
done
