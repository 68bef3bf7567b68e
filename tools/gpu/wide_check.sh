# Wide engine: tests, skinny phase stamps, bench, per-kernel stats.  Usage: bash tools/gpu/wide_check.sh TAG
set -e
T=${1:-wc}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_skinny.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 120 python tools/skinny_stamps.py gpurun_out/${T}_skinny.json > /dev/null 2> gpurun_out/${T}_skinny.err && python -c "
import json; d=json.load(open('gpurun_out/${T}_skinny.json'))
for k,v in d.items(): print(k, v)"
timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/${T}_wide.json 2> gpurun_out/${T}_wide.err && cut -c1-160 gpurun_out/${T}_wide.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python $GRAFT_REPO_ROOT/bench_wide.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 && cd $GRAFT_REPO_ROOT && python tools/rocpd_summary.py gpurun_out/${T}_prof/run_results.db --skip 200 | cut -c1-150
