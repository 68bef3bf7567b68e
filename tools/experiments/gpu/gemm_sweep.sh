set -e
mkdir -p gpurun_out
python -c "import hipdsml._build as b; b.build()" > gpurun_out/build.log 2>&1
for f in 0 1 2 3; do HIPDSML_R64_FLAGS=$f timeout -k 10 120 python tools/gemm_bench.py >> gpurun_out/gemm_sweep.jsonl; done
cat gpurun_out/gemm_sweep.jsonl
