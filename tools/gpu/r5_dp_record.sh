# Round-5 data-parallel record on one MI355X: the lone-replica probe of every
# persistent form at N = 1/2/4/8 (one box, so the ratios to N = 1 compare), the
# 2-rank rehearsal (2 processes sharing the GPU, sync=auto and pkx), and the
# single-replica bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_dp
mkdir -p $O
for al in 4 2 0; do
  timeout -k 10 200 python $R/tools/pk_probe.py --algo $al --ranks 1,2,4,8 --steps 2000 > $O/probe_algo$al.jsonl 2>&1
done
timeout -k 10 300 python $R/bench.py --gpus 2 --rehearse-one-gpu --steps 2000 --warmup 200 --no-allreduce-probe > $O/rehearse2_auto.json 2> $O/rehearse2_auto.err
timeout -k 10 300 python $R/bench.py --gpus 2 --rehearse-one-gpu --steps 2000 --warmup 200 --sync pkx --no-allreduce-probe --no-sync-sweep > $O/rehearse2_pkx.json 2> $O/rehearse2_pkx.err
timeout -k 10 100 python $R/bench.py --steps 2000 --warmup 200 --no-e2e > $O/bench_n1_2000.json 2>/dev/null
timeout -k 10 100 python $R/bench.py --steps 20 --warmup 5 > $O/bench_n1_driver.json 2>/dev/null
