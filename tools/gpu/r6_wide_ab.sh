# Wide step with the consumer-combined split-K GEMMs: tests, then bench_wide
# alternating head slabs 0 / 1 (dgrad slabs were removed), then a kernel
# trace of the default (both on).
set -e
T=${1:-r6w}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_gemm_skinny.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
for k in 1 2; do
  for hd in "0 0" "1 0"; do
    set -- $hd
    HIPDSML_WIDE_HEAD_SLABS=$1 HIPDSML_WIDE_DGRAD_SLABS=$2 timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 2>/dev/null > gpurun_out/${T}_bench_$1$2_$k.json
    echo "head=$1 dgrad=$2 $(cut -c1-110 gpurun_out/${T}_bench_$1$2_$k.json)"
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${T}_prof -o run -- python $GRAFT_REPO_ROOT/bench_wide.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log 2>&1 && cd $GRAFT_REPO_ROOT && python tools/rocpd_summary.py gpurun_out/${T}_prof/run_results.db --skip 200 --csv gpurun_out/${T}_kernels.csv | cut -c1-150
