# Flagship N=1: repeat the headline bench and take a rocprofv3 kernel trace.
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for i in 1 2 3; do timeout -k 10 120 python bench.py > gpurun_out/b$i.json 2>/dev/null; python -c "import json;d=json.load(open('gpurun_out/b$i.json'));print('bench', d['ms_per_step'])"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_n1 -o run -- python3 $R/bench.py --steps 2000 --warmup 200 > $R/gpurun_out/prof_n1.log 2>&1
cd $R && find gpurun_out/prof_n1 -name "*.db" | head -1 | xargs -I{} python tools/rocpd_summary.py {} --skip 1000 --csv gpurun_out/prof_n1_kernels.csv | head -12
