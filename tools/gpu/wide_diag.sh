# Wide engine diagnostics: head phases, skinny GEMM phase stamps, isolated GEMM
# timings, the step's per-kernel stats.  Usage: bash tools/gpu/wide_diag.sh TAG
set -e
T=${1:-wd}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python tools/experiments/head_bench.py > gpurun_out/${T}_head.json 2> gpurun_out/${T}_head.err && cat gpurun_out/${T}_head.json
timeout -k 10 120 python tools/skinny_stamps.py gpurun_out/${T}_skinny.json > /dev/null 2> gpurun_out/${T}_skinny.err && python -c "
import json; d=json.load(open('gpurun_out/${T}_skinny.json'))
for k,v in d.items(): print(k, v)"
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/${T}_gemm.json 2> gpurun_out/${T}_gemm.err && cat gpurun_out/${T}_gemm.json
timeout -k 10 200 python bench_wide.py --steps 200 --warmup 20 > gpurun_out/${T}_wide.json 2> gpurun_out/${T}_wide.err && cut -c1-200 gpurun_out/${T}_wide.json
