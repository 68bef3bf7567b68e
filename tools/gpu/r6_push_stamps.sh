# pkx mirror mode (the one-GPU estimate of the real protocol): pusher-0 and
# tile-0 gather timeline at N = 4 / 8 from the measurement build
set -e -o pipefail
O=gpurun_out/${1:-r6push}
mkdir -p $O
SO=distributed-machine-learning-pipeline_amd/_C.so
cp $SO $O/prod_C.so
cp tools/measure_so/_C.so $SO
timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 4,8 --mirror --stamps $O/st.jsonl --push-stamps $O/push.jsonl > $O/probe.txt 2> $O/err.txt || { cp $O/prod_C.so $SO; tail -5 $O/err.txt; exit 1; }
cp $O/prod_C.so $SO
cut -c1-110 $O/probe.txt
cat $O/push.jsonl
