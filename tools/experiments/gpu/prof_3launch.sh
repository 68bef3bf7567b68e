# Per-kernel times of the three-launch step (the N > 1 path) on one GPU.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
HIPDSML_PERSIST=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_3l -o run -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/prof_3l.log 2>&1
cd $R && find gpurun_out/prof_3l -name "*.db" | head -1 | xargs -I{} python tools/rocpd_summary.py {} --csv gpurun_out/prof_3l_kernels.csv | head -8
