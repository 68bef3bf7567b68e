# pkx lone-replica probe with the placement search the DP bench uses (4
# hand-off buffers, fastest kept): HEAD~ (old) vs the correction + tagged
# partials change (new), alternating .so swaps
set -e
SO=distributed-machine-learning-pipeline_amd/_C.so
for k in 1 2 3; do
  for v in old new; do
    cp abso/C_$v.so $SO
    timeout -k 10 200 python tools/pk_probe.py --algo 4 --ranks 2,4,8 --place 4 2>/dev/null | cut -c1-130 | sed "s/^/$v /"
  done
done
cp abso/C_new.so $SO
