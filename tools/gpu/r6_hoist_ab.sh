# pkx: DZR pointers hoisted out of the poll rounds + the helpers' probe pacing
# merged into their poll rounds (new4) vs the committed tree (new); placement
# search as the DP bench; then the persist tests on new4
set -e
O=gpurun_out/${1:-r6hoist}
mkdir -p $O
SO=distributed-machine-learning-pipeline_amd/_C.so
for k in 1 2 3; do
  for v in new new4; do
    cp abso/C_$v.so $SO
    timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 2,4,8 --place 4 2>/dev/null | cut -c1-130 | sed "s/^/$v /"
    timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 8 --mirror 2>/dev/null | cut -c1-100 | sed "s/^/$v mirror /"
  done
done
cp abso/C_new4.so $SO
timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 8 --place 4 --stamps $O/st_new4.jsonl > /dev/null 2>$O/err.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
