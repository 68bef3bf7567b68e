# Merged local + peer dZ1 poll in the Gram-form layer-1 blocks: tests, then the
# lone-replica probe (pkx, pkg) of the staged old / new builds alternating, the
# 2-rank rehearsal and the single-replica bench of the new tree.
set -e
T=${1:-dz}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_dp.py tests/test_gpu_xchg.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 1 2; do
  for v in old new; do
    for al in 4 2; do
      echo -n "$v algo$al "; (cd abtmp/$v && timeout -k 10 200 python tools/pk_probe.py --algo $al --ranks 1,2,4,8 --steps 2000 --place 3 2>/dev/null) | python -c "
import json,sys
r={}
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); r[d['ranks']]=d['us_per_step']
print(r, {k: round(v/r[1],3) for k,v in r.items()} if 1 in r else '')"
    done
  done
done
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 2000 --warmup 200 --sync pkx --no-allreduce-probe --no-sync-sweep > gpurun_out/${T}_reh2.json 2> gpurun_out/${T}_reh2.err
cut -c1-200 gpurun_out/${T}_reh2.json
