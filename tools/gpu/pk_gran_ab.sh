# Data-parallel persistent step: flag protocol vs granule protocol (HIPDSML_PK_GRAN), 2/3-process IPC
# tests under each, and 2-rank one-GPU rehearsals with sync=pk.
set -e
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_xchg.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_xchg.log 2>&1 || { tail -30 gpurun_out/pytest_xchg.log; exit 1; }
echo "xchg suite: $(tail -1 gpurun_out/pytest_xchg.log)"
for g in 1 0; do
  HIPDSML_PK_GRAN=$g timeout -k 10 300 python -u -m pytest tests/test_gpu_xchg.py -m gpu -x -q --timeout 150 --timeout-method thread -k "pk" > gpurun_out/pytest_pk_g$g.log 2>&1 || { tail -30 gpurun_out/pytest_pk_g$g.log; exit 1; }
  echo "gran=$g $(tail -1 gpurun_out/pytest_pk_g$g.log)"
  HIPDSML_PK_GRAN=$g timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --sync pk --steps 1000 --warmup 100 --no-sync-sweep > gpurun_out/pk2_g$g.json 2> gpurun_out/pk2_g$g.err
  echo "gran=$g $(python -c "import json;d=json.load(open('gpurun_out/pk2_g$g.json'));print(d['ms_per_step'], d['config']['sync'])")"
done
timeout -k 10 200 python tools/pk_dp_stamps.py gpurun_out/pk_dp_stamps_g0.json > gpurun_out/pk_dp_stamps.log 2>&1 && cat gpurun_out/pk_dp_stamps_g0.json
