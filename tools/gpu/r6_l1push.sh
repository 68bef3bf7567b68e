# pkx dZ1 row pushes from the chains (l1push 0) or the layer-1 owner blocks (1):
# the replay / mirror tests with both, then alternating mirror-mode and
# lone-probe step times at N = 4 / 8, and stamps of both.
set -e
O=gpurun_out/${1:-r6f}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py -k "replay or mirrored" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in 1 2; do
  for p in 0 1; do
    timeout -k 10 200 python tools/pk_probe.py --mirror --algo 4 --ranks 4,8 --steps 2000 --l1push $p >> $O/mirror.jsonl 2>> $O/probe.err
    timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 4,8 --steps 2000 --l1push $p >> $O/probe.jsonl 2>> $O/probe.err
  done
done
for p in 0 1; do
  timeout -k 10 200 python tools/pk_probe.py --mirror --algo 4 --ranks 8 --steps 2000 --l1push $p --stamps $O/stamps.jsonl > /dev/null 2>> $O/probe.err
done
cat $O/mirror.jsonl $O/probe.jsonl
