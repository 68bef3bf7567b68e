# pkx / pkg: speculative partial gather (first look by LDS-DMA before the dZ1
# poll, the rest after it; new5) vs the hoist + pacing tree (new4); placement
# search as the DP bench; then the persist tests on new5
set -e -o pipefail
O=gpurun_out/${1:-r6spec}
mkdir -p $O
SO=distributed-machine-learning-pipeline_amd/_C.so
cp abso/C_new5.so $SO
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2 3; do
  for v in new4 new5; do
    cp abso/C_$v.so $SO
    timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 2,4,8 --place 4 2>/dev/null | cut -c1-130 | sed "s/^/$v /"
    timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 8 --mirror 2>/dev/null | cut -c1-100 | sed "s/^/$v mirror /"
  done
done
cp abso/C_new5.so $SO
timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 8 --place 4 --stamps $O/st_new5.jsonl > /dev/null 2>$O/err.txt
