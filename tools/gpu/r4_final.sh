# Round-4 final evidence (phase a: suite .. rehearsals; phase b: profiles,
# wide, RPC).  The driver's round-end steps (suite, smoke, bench in
# driver form), then the profiles the README cites.  Every GPU step bounded.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
T=${1:-r4f}
PH=${2:-a}
if [ "$PH" = a ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_suite.log 2>&1 || { tail -60 gpurun_out/${T}_suite.log; exit 1; }
tail -2 gpurun_out/${T}_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 && tail -1 gpurun_out/${T}_smoke.log
for k in 1 2 3; do timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench20_$k.json 2>/dev/null; cut -c1-160 gpurun_out/${T}_bench20_$k.json; done
timeout -k 10 200 python bench.py --gpus 1 --steps 2000 --warmup 200 > gpurun_out/${T}_bench2000.json 2>/dev/null && cut -c1-160 gpurun_out/${T}_bench2000.json
timeout -k 10 120 python tools/pk_stamps.py gpurun_out/${T}_stamps.json > /dev/null 2>&1
timeout -k 10 300 python tools/pk_overhead.py gpurun_out/${T}_overhead.json > /dev/null 2>&1
for al in 0 1 2 3 4; do timeout -k 10 200 python tools/pk_probe.py --algo $al --steps 2000 > gpurun_out/${T}_probe_$al.jsonl 2>/dev/null; done
cat gpurun_out/${T}_probe_*.jsonl | cut -c1-120
for m in pkx pkg pk auto; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29742 bench.py --gpus 2 --steps 2000 --warmup 200 --sync $m --rehearse-one-gpu > gpurun_out/${T}_reh2_$m.json 2>/dev/null
  grep -v Gloo gpurun_out/${T}_reh2_$m.json | cut -c1-200 || true
done
exit 0
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/${T}_prof.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_p1 -o run --output-format csv -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/${T}_p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/${T}_p2 -o run --output-format csv -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/${T}_p2.log 2>&1
cd $R
python tools/pmc_summary.py gpurun_out/${T}_pmc.json persist=mlp_persist_k:gpurun_out/${T}_p1,gpurun_out/${T}_p2 > /dev/null
DB=$(find gpurun_out/${T}_prof -name "*.db" | sort | tail -n 1)
python tools/rocpd_summary.py $DB --csv gpurun_out/${T}_kernels.csv > gpurun_out/${T}_kernels.txt && cut -c1-160 gpurun_out/${T}_kernels.csv | sed -n 1,4p
timeout -k 10 300 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/${T}_wide.json 2>/dev/null && cut -c1-200 gpurun_out/${T}_wide.json
bash tools/gpu/rpc_ar.sh
timeout -k 10 400 python -m hipdsml.bench.train_rpc --devices 2 --steps 50,937 --reps 5 --out gpurun_out/${T}_rpc_n2.json > /dev/null 2>&1 && cut -c1-400 gpurun_out/${T}_rpc_n2.json
