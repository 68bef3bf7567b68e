# (the HIPDSML_PK_PUSH_AUX knob was removed after this A/B: no effect)
# pkx mirror mode, measurement build: the pushers' store cache policy
# (HIPDSML_PK_PUSH_AUX 0 system scope sc0|sc1 = production, 1 sc1, 2 plain)
# -- step time and the pusher-0 timeline at N = 4 / 8
set -e -o pipefail
O=gpurun_out/${1:-r6pushaux}
mkdir -p $O
SO=distributed-machine-learning-pipeline_amd/_C.so
cp $SO $O/prod_C.so
cp tools/measure_so/_C.so $SO
for k in 1 2; do
  for x in 0 1 2; do
    HIPDSML_PK_PUSH_AUX=$x timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 4,8 --mirror --stamps $O/st_$x.jsonl --push-stamps $O/push_$x.jsonl > $O/probe_${x}_$k.txt 2> $O/err_$x.txt || { cp $O/prod_C.so $SO; tail -5 $O/err_$x.txt; exit 1; }
    cut -c1-100 $O/probe_${x}_$k.txt | sed "s/^/aux=$x /"
  done
done
cp $O/prod_C.so $SO
for x in 0 1 2; do sed "s/^/aux=$x /" $O/push_$x.jsonl; done
