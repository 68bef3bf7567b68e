# Persistent-step chain placement A/B (HIPDSML_PK_PLACE 0 / 1), plus the wide and persistent GPU tests.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_persist.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1 || { tail -30 gpurun_out/pytest_sub.log; exit 1; }
tail -1 gpurun_out/pytest_sub.log
for r in 1 2; do for p in 0 1; do
  HIPDSML_PK_PLACE=$p timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/pl${p}_20_$r.json 2>/dev/null
  HIPDSML_PK_PLACE=$p timeout -k 10 120 python bench.py --steps 2000 --warmup 200 > gpurun_out/pl${p}_2000_$r.json 2>/dev/null
  echo "place=$p run=$r $(python -c "import json;print(json.load(open('gpurun_out/pl${p}_20_$r.json'))['ms_per_step'], json.load(open('gpurun_out/pl${p}_2000_$r.json'))['ms_per_step'])")"
done; done
