# pkx / single replica: tagged-granule layer-1 partials (pg) vs flag + drain
# (corr: correction change only) vs HEAD (old); .so swap A/B, then the persist
# tests and the N = 1 bench on the new build
set -e
O=gpurun_out/${1:-r6pg}
mkdir -p $O
SO=distributed-machine-learning-pipeline_amd/_C.so
for k in 1 2 3; do
  for v in old corr new2; do
    cp abso/C_$v.so $SO
    timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 1,2,4,8 2>/dev/null | cut -c1-100 | sed "s/^/$v probe /"
  done
done
for v in old new2 old new2; do
  cp abso/C_$v.so $SO
  timeout -k 10 200 python bench.py --steps 2000 --warmup 200 2>/dev/null | cut -c1-140 | sed "s/^/$v bench2000 /"
done
cp abso/C_new2.so $SO
timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 1,8 --stamps $O/st_new2.jsonl > /dev/null 2>$O/err.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
