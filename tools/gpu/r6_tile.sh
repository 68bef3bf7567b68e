# Wide step: the update of the layers above the input layer on 64x64 vs 128x128 tiles
set -e
O=gpurun_out/${1:-r6tile}
R=$GRAFT_REPO_ROOT
mkdir -p $O
for k in 1 2; do
  for t in 0 128; do
    HIPDSML_WIDE_WG_TILE=$t timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > $O/ab_${t}_$k.json 2>/dev/null
    echo "tile=$t $(cut -c1-140 $O/ab_${t}_$k.json)"
  done
done
cd /tmp && export TMPDIR=/tmp && HIPDSML_WIDE_WG_TILE=128 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/$O/wprof -o run -- python $R/bench_wide.py --steps 100 --warmup 10 > $R/$O/wprof.log 2>&1 && cd $R && python tools/rocpd_summary.py $O/wprof/run_results.db --skip 200 --csv $O/wide_kernels.csv | cut -c1-150
