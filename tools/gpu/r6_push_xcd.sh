# pkx mirror mode, measurement build: pusher-0 timeline with the pushers on
# XCD 0 beside the gradient tiles (3 helpers, default) vs in the layer-1 XCDs'
# spare CUs (HIPDSML_PKX_HELPERS=1 moves them there; the dW1 split changes too)
set -e -o pipefail
O=gpurun_out/${1:-r6pushxcd}
mkdir -p $O
SO=distributed-machine-learning-pipeline_amd/_C.so
cp $SO $O/prod_C.so
cp tools/measure_so/_C.so $SO
for k in 1 2; do
  for h in 3 1; do
    HIPDSML_PKX_HELPERS=$h timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 8 --mirror --stamps $O/st_$h.jsonl --push-stamps $O/push_$h.jsonl > $O/probe_${h}_$k.txt 2> $O/err_$h.txt || { cp $O/prod_C.so $SO; tail -5 $O/err_$h.txt; exit 1; }
    cut -c1-100 $O/probe_${h}_$k.txt | sed "s/^/helpers=$h /"
  done
done
cp $O/prod_C.so $SO
for h in 3 1; do sed "s/^/helpers=$h /" $O/push_$h.jsonl; done
