# Round 6 final check (after the pkx layer-1 changes): every GPU test, smoke, the
# headline bench, the wide bench + kernel trace, the row-block PMC, the lone-replica probe and the 2-rank rehearsal.
set -e -o pipefail
T=${1:-r6final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && cat $O/smoke.log
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err
timeout -k 10 120 python bench.py --no-e2e > $O/bench2000.json 2> $O/bench2000.err
cut -c1-200 $O/bench20.json $O/bench2000.json
for k in 1 2; do timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 2>/dev/null | cut -c1-120; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/wprof -o run -- python $GRAFT_REPO_ROOT/bench_wide.py --steps 100 --warmup 10 > $GRAFT_REPO_ROOT/$O/wprof.log 2>&1 && cd $GRAFT_REPO_ROOT && python tools/rocpd_summary.py $O/wprof/run_results.db --skip 200 --csv $O/wide_kernels.csv | cut -c1-150
bash tools/gpu/r6_rb_pmc.sh $T/rb
timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 1,2,4,8 --place 4 > $O/probe.txt 2>/dev/null && cut -c1-110 $O/probe.txt
timeout -k 10 400 python bench.py --gpus 2 --rehearse-one-gpu --steps 200 --warmup 50 > $O/n2.json 2> $O/n2.err && tail -1 $O/n2.json | cut -c1-300
