# Price of idle workgroups in the single-replica persistent launch: extra idle
# blocks (HIPDSML_PK_GRID_EXTRA) against none, alternating, 2,000 steps and the
# driver's 20-step form.
# Needs the measurement build (the knob is compiled out of production builds):
#   python -m hipdsml._build --measure   (then python -m hipdsml._build to restore)
set -e
mkdir -p gpurun_out
python -c "import hipdsml.ops.native as n; assert n.require_native().measure_build, 'build with --measure'"
for k in 1 2; do
  for x in 0 48 96; do
    for S in "2000 200" "20 5"; do
      set -- $S
      HIPDSML_PK_GRID_EXTRA=$x timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-e2e 2>/dev/null \
        | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('extra=$x steps=$1', d['ms_per_step']*1000)" | tee -a gpurun_out/gx_ab.txt
    done
  done
done
