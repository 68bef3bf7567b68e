# Kernel stats of the in-process 2-replica run: activation vs gradient exchange.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for m in xact xgmi; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_local_$m -o run -- python3 $R/tools/xchg_local_bench.py --replicas 2 --steps 1000 --mode $m > $R/gpurun_out/prof_local_$m.log 2>&1
done
cat $R/gpurun_out/prof_local_*.log | grep replicas
find $R/gpurun_out/prof_local_* -name "*kernel_stats.csv"
