# Instruction-cache counters of the persistent step: single replica and the
# pkx lone-replica probe at 8 replicas (one pass each, kernel-trace only).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_ic1 $R/gpurun_out/pmc_ic8
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES --kernel-trace -d $R/gpurun_out/pmc_ic1 -o run -- python3 $R/tools/pk_probe.py --algo 4 --ranks 1 --steps 2000 > $R/gpurun_out/pmc_ic1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES --kernel-trace -d $R/gpurun_out/pmc_ic8 -o run -- python3 $R/tools/pk_probe.py --algo 4 --ranks 8 --steps 2000 > $R/gpurun_out/pmc_ic8.log 2>&1
python3 $R/tools/pmc_summary.py $R/gpurun_out/r5_pmc_icache.json n1=mlp_persist_k:$R/gpurun_out/pmc_ic1 n8=mlp_persist_k:$R/gpurun_out/pmc_ic8
