# rocprofv3 kernel summaries of the flagship step, the wide step and the
# in-process xGMI exchange (single-process runs only).
set -e
mkdir -p gpurun_out
python -c "import hipdsml._build as b; b.build()" > gpurun_out/build.log 2>&1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_n1 -o run -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/prof_n1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wide -o run -- python3 $R/bench_wide.py --steps 50 --warmup 5 > $R/gpurun_out/prof_wide.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_xchg -o run -- python3 $R/tools/xchg_local_bench.py --replicas 2 --steps 1000 > $R/gpurun_out/prof_xchg.log 2>&1
timeout -k 10 120 python3 $R/tools/xchg_local_bench.py --replicas 2 --steps 2000 > $R/gpurun_out/xchg_local2.json
timeout -k 10 120 python3 $R/tools/xchg_local_bench.py --replicas 3 --steps 2000 > $R/gpurun_out/xchg_local3.json
cat $R/gpurun_out/xchg_local*.json
find $R/gpurun_out/prof_* -name "*kernel_stats.csv" | head
