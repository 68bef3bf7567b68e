# Round-2 full check: GPU tests, smoke, N=1 bench (driver form + default), rocprof of the
# default bench (persistent step), 2-rank self-launched rehearsal.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.err && cat gpurun_out/bench20.json
timeout -k 10 200 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
HIPDSML_PERSIST=0 timeout -k 10 200 python bench.py > gpurun_out/bench_3launch.json 2>/dev/null && cat gpurun_out/bench_3launch.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pk -o run -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/prof_pk.log 2>&1
cd $R && find gpurun_out/prof_pk -name "*.db" | head -1 | xargs -I{} python tools/rocpd_summary.py {} --csv gpurun_out/prof_pk_kernels.csv | head -8
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 1000 --warmup 100 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err && cat gpurun_out/rehearse2.json
