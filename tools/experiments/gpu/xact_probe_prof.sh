# Per-kernel times of the lone-replica sync probe (tools/xact_probe.py) at N = 2 and 8.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for n in 2 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_probe$n -o run -- python3 $R/tools/xact_probe.py --ranks $n --steps 1000 > $R/gpurun_out/prof_probe$n.log 2>&1
done
