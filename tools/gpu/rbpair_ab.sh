# Row-block update with two ring blocks per wait / barrier: the row-block and
# DP tests on the new tree, then the global-batch update cost of the staged
# old (one block) / new (pairs) builds, alternating, with and without traffic.
# The no-traffic rows need measurement builds of both trees (HIPDSML_RB_DBG is
# compiled out of production builds): python -m hipdsml._build --measure.
set -e
T=${1:-rp}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_skinny.py -k "rowblk or wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_dp.log 2>&1 || { tail -40 gpurun_out/${T}_dp.log; exit 1; }
tail -1 gpurun_out/${T}_dp.log
for k in 1 2; do
  for v in old new; do
    echo -n "$v "; (cd abtmp/$v && timeout -k 10 200 python tools/wide_xact_cost.py 2>/dev/null | cut -c1-110)
  done
done
for v in old new; do
  echo -n "$v no-traffic "; (cd abtmp/$v && HIPDSML_RB_DBG=7 timeout -k 10 200 python tools/wide_xact_cost.py 2>/dev/null | cut -c1-110)
done
