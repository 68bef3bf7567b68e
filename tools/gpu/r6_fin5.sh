# after the pkx correction / tagged-partials change: every GPU test, smoke,
# the headline bench (driver form and 2,000 steps), the lone-replica probe and
# the 2-rank one-GPU rehearsal
set -e
O=gpurun_out/${1:-r6fin5}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -40 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && cat $O/smoke.log
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err
timeout -k 10 120 python bench.py --no-e2e > $O/bench2000.json 2> $O/bench2000.err
cut -c1-200 $O/bench20.json $O/bench2000.json
for k in 1 2; do timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 1,2,4,8 2>/dev/null | cut -c1-100; done
timeout -k 10 400 python bench.py --gpus 2 --rehearse-one-gpu --steps 200 --warmup 50 > $O/n2.json 2> $O/n2.err
tail -1 $O/n2.json | cut -c1-400
