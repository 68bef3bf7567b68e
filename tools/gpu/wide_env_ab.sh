# A/B of one wide-engine switch: tests matching a pattern, benches alternating
# VAR=0 / VAR=1, then a kernel trace with VAR=1.
#   bash tools/gpu/wide_env_ab.sh TAG VAR PYTEST_K
set -e
T=$1; V=$2; K=$3
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -q -k "$K" --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 1 2; do
  for f in 0 1; do
    env $V=$f timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 2>/dev/null > gpurun_out/${T}_bench_${f}_$k.json
    echo "$V=$f $(cut -c1-110 gpurun_out/${T}_bench_${f}_$k.json)"
  done
done
export $V=1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python $GRAFT_REPO_ROOT/bench_wide.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 && cd $GRAFT_REPO_ROOT && python tools/rocpd_summary.py gpurun_out/${T}_prof/run_results.db --skip 200 --csv gpurun_out/${T}_kernels.csv | cut -c1-150
