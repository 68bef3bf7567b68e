# pkx layer-1 correction: LDS operands read up front + LDS-only barriers after
# the dZ1 poll (new) vs per-replica reads + __syncthreads (old); .so swap A/B
set -e
O=gpurun_out/${1:-r6corr}
mkdir -p $O
SO=distributed-machine-learning-pipeline_amd/_C.so
for k in 1 2 3; do
  for v in old new; do
    cp abso/C_$v.so $SO
    timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 2,4,8 2>/dev/null | cut -c1-100 | sed "s/^/$v probe /"
  done
done
cp abso/C_new.so $SO
timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 2,8 --stamps $O/st_new.jsonl > /dev/null 2>$O/err.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -k "replay or mirrored or bit_exact" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
