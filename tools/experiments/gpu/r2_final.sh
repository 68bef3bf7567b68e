# Round-2 final evidence: GPU suite, smoke, driver-form + default N=1 bench, wide bench,
# rocprof kernel stats of the default bench (persistent step) and of the wide bench.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.json 2> gpurun_out/bench20.err && cat gpurun_out/bench20.json
timeout -k 10 200 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json
timeout -k 10 300 python bench_wide.py > gpurun_out/bench_wide.json 2> gpurun_out/bench_wide.err && cat gpurun_out/bench_wide.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pk -o run -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/prof_pk.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wide -o run -- python3 $R/bench_wide.py --steps 50 --warmup 5 > $R/gpurun_out/prof_wide.log 2>&1
cd $R && ls -R gpurun_out/prof_pk | head -20
