# gpu_sim AllReduceRing dispatch: gRPC futures fan-out vs the thread pool
# (HIPDSML_COORD_FUTURES), 3 device servers, 1 MiB, host and hip devices.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in hip host; do
  for k in 1 2; do
    for t in 0 1; do
      HIPDSML_COORD_FUTURES=$t timeout -k 10 300 python -m hipdsml.bench.allreduce rpc --backend $b --reps 30 > gpurun_out/cf_${b}_t${t}_$k.json 2>/dev/null
      echo "$b futures=$t $(python -c "import json; d=json.loads(open('gpurun_out/cf_${b}_t${t}_$k.json').read().splitlines()[-1]); print(d['ring_as_published_ms_median'], d['ring_full_fp32_ms_median'], d['ring_per_segment_rpc_fp32_ms_median'], d.get('xgmi_fp32_ms_median'), d['naive_ms_median'])")"
    done
  done
done
