# Round 6: the replay test of the data-parallel persistent forms on distinct
# peer data, the RPC / pg / fit GPU tests, the bench, the RPC all-reduce, then
# (measurement build, copied in last) the hop-latency sweep in mirror mode.
set -e
O=gpurun_out/${1:-r6c}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py -k "replay" -x -v --timeout 120 --timeout-method thread > $O/replay.log 2>&1 || { tail -30 $O/replay.log; exit 1; }
tail -3 $O/replay.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_rpc.py tests/test_pg_bootstrap.py tests/test_gpu_fit.py -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 180 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -m hipdsml bench-allreduce rpc --n 3 --backend hip > $O/ar_rpc3.json 2> $O/ar_rpc3.err
cp tools/measure_so/_C.so distributed-machine-learning-pipeline_amd/_C.so
for algo in 4 2 0; do
  timeout -k 10 200 python tools/pk_probe.py --mirror --algo $algo --ranks 4,8 --steps 2000 --hop-us 0,1,2,4 >> $O/hop.jsonl 2> $O/hop_$algo.err
done
cat $O/hop.jsonl
