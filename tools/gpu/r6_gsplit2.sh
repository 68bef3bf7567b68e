# pkx dW1 split: 1 (gatherer owners take no replica) vs 2 (no owner takes one), replay test for 2
set -e
O=gpurun_out/${1:-r6gsplit2}
mkdir -p $O
HIPDSML_PKX_GSPLIT=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py -k "replay" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for f in 1 2; do
    HIPDSML_PKX_GSPLIT=$f timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 4,8 2>/dev/null | cut -c1-100 | sed "s/^/gsplit=$f probe /"
    HIPDSML_PKX_GSPLIT=$f timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 8 --mirror 2>/dev/null | cut -c1-100 | sed "s/^/gsplit=$f mirror /"
  done
done
