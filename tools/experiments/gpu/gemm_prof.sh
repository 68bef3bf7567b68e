# Kernel durations of the GEMM microbenchmark (rocprofv3 kernel trace).
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_gemm -o run -- python3 $R/tools/gemm_bench.py --iters 20 > $R/gpurun_out/prof_gemm.log 2>&1
