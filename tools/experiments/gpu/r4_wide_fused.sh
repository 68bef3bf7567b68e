# Fused wide backward (wide_bwd): tests, bench A/B (separate dgrad vs fused at
# several slice heights), kernel trace of the default.  Usage: bash tools/gpu/wide_fused.sh TAG
set -e
T=${1:-wf}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
HIPDSML_WIDE_FUSED_BWD=0 timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/${T}_wide_sep.json 2>/dev/null && cut -c1-120 gpurun_out/${T}_wide_sep.json
for sp in 1; do for r in 512 1024; do
  HIPDSML_WIDE_BWD_SPLIT=$sp HIPDSML_WIDE_BWD_ROWS=$r timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/${T}_wide_s${sp}_r$r.json 2>/dev/null && cut -c1-120 gpurun_out/${T}_wide_s${sp}_r$r.json | sed "s/^/split $sp rows $r /"
done; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python $GRAFT_REPO_ROOT/bench_wide.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 && cd $GRAFT_REPO_ROOT && python tools/rocpd_summary.py gpurun_out/${T}_prof/run_results.db --skip 200 --csv gpurun_out/${T}_kernels.csv | cut -c1-150
