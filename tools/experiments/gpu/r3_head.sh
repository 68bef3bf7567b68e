set -e
mkdir -p gpurun_out
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 120 python tools/experiments/head_bench.py > gpurun_out/r3h_head.json 2> gpurun_out/r3h_head.err && cat gpurun_out/r3h_head.json
