# pkx pushers: the slot data registers pinned across the peer loop (pin: no
# re-materialized tag lanes rewriting the data of stores in flight) vs the
# previous tree (old); mirror mode and the probe at N = 4 / 8, alternating
# .so swaps; then the pusher timeline (measurement build, pin) and the tests
set -e -o pipefail
O=gpurun_out/${1:-r6pin}
mkdir -p $O
SO=distributed-machine-learning-pipeline_amd/_C.so
for k in 1 2 3; do
  for v in old pin; do
    cp abso/C_$v.so $SO
    timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 4,8 --mirror 2>/dev/null | cut -c1-100 | sed "s/^/$v mirror /"
    timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 8 --place 4 2>/dev/null | cut -c1-100 | sed "s/^/$v probe /"
  done
done
cp tools/measure_so/_C.so $SO
timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 8 --mirror --push-stamps $O/push.jsonl --stamps $O/st.jsonl > /dev/null 2> $O/err.txt || { cp abso/C_pin.so $SO; tail -5 $O/err.txt; exit 1; }
cat $O/push.jsonl
cp abso/C_pin.so $SO
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
