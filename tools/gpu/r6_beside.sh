# Input-layer strips inside the update launch: tests, A/B (own launch vs beside), trace
set -e
T=${1:-r6beside}
R=$GRAFT_REPO_ROOT
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 120 --timeout-method thread -k "fused_input" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2; do
  for f in 0 1; do
    HIPDSML_WIDE_INPUT_BESIDE=$f timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > $O/ab_${f}_$k.json 2>/dev/null
    echo "beside=$f $(cut -c1-140 $O/ab_${f}_$k.json)"
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/wprof -o run -- python $R/bench_wide.py --steps 100 --warmup 10 > $R/$O/wprof.log 2>&1 && cd $R && python tools/rocpd_summary.py $O/wprof/run_results.db --skip 200 --csv $O/wide_kernels.csv | cut -c1-150
