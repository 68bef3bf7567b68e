# Hand-off buffer placement autotune on/off (HIPDSML_PK_PLACE=1 vs default),
# alternating bench.py runs on one box: 2000-step and the driver's 20-step form.
set -e
T=${1:-pl}
mkdir -p gpurun_out
for k in 1 2 3 4; do
  for v in 1 8; do
    for S in "2000 200" "20 5"; do
      set -- $S
      HIPDSML_PK_PLACE=$v timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-e2e 2>/dev/null \
        | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('place=$v steps=$1', d['ms_per_step']*1000, d['config']['precompute'].get('persist_place_us'))" | tee -a gpurun_out/${T}_ab.txt
    done
  done
done
