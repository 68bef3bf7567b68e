# A/B of two builds staged by hand under abtmp/{old,new} (each: bench.py + a
# full hipdsml copy with its own _C.so): alternating runs on one box.
# usage: ab_bench.sh TAG STEPS WARMUP ROUNDS [extra bench args]
set -e
T=$1; S=$2; W=$3; N=$4; shift 4
mkdir -p gpurun_out
for k in $(seq 1 $N); do
  for v in old new; do
    (cd abtmp/$v && timeout -k 10 200 python bench.py --steps $S --warmup $W --no-e2e "$@" 2>/dev/null) | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step']*1000)" | tee -a gpurun_out/${T}_ab.txt
  done
done
