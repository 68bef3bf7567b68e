set -e
mkdir -p gpurun_out
python -c "import hipdsml._build as b; b.build()" > gpurun_out/build.log 2>&1
timeout -k 10 120 python tools/gemm_probe.py > gpurun_out/gemm_probe.json
cat gpurun_out/gemm_probe.json
