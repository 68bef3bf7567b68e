# pkx: gatherer-tile owners leave every dW1 replica to their helpers (HIPDSML_PKX_GSPLIT 1) vs
# the even split (0): the replay test on distinct peers with the split on, then the
# lone-replica probe and mirror mode at N = 4 / 8, alternating
set -e
O=gpurun_out/${1:-r6gsplit}
mkdir -p $O
HIPDSML_PKX_GSPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py -k "replay or mirror" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for f in 0 1; do
    HIPDSML_PKX_GSPLIT=$f timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 4,8 2>/dev/null | cut -c1-100 | sed "s/^/gsplit=$f probe /"
    HIPDSML_PKX_GSPLIT=$f timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 4,8 --mirror 2>/dev/null | cut -c1-100 | sed "s/^/gsplit=$f mirror /"
  done
done
