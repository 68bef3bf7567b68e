# RPC-level naive-vs-ring experiment (BASELINE metric 2, view (a)) on GPU and
# host device servers, 3 processes each.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m hipdsml.bench.allreduce rpc --n 3 --backend hip --reps 15 > gpurun_out/r4_allreduce_rpc_hip.json 2> gpurun_out/rpc_ar_hip.err
cat gpurun_out/r4_allreduce_rpc_hip.json
timeout -k 10 300 python -m hipdsml.bench.allreduce rpc --n 3 --backend host --reps 15 --base-port 6303 > gpurun_out/r4_allreduce_rpc_host.json 2> gpurun_out/rpc_ar_host.err
cat gpurun_out/r4_allreduce_rpc_host.json
