# Fused input layer: phase stamps with load kinds dropped (measurement build)
set -e
O=gpurun_out/${1:-r6widbg}
mkdir -p $O
cp tools/measure_so/_C.so distributed-machine-learning-pipeline_amd/_C.so
for d in 0 1 2 3 4 8 15; do
  WI_DBG=$d timeout -k 10 120 python tools/wide_input_stamps.py > $O/stamps_$d.json 2> $O/err_$d.log
  cut -c1-400 $O/stamps_$d.json
done
