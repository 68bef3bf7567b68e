# (knob HIPDSML_PK_OWNLAST since removed: no difference) pkx merged dZ1 poll: this replica's own rows loaded first (0) or after the
# peers' (1) in each poll round; lone-replica probe at N = 2/4/8 alternating,
# plus one stamped run each (correction split stamps)
set -e
O=gpurun_out/${1:-r6ownlast}
mkdir -p $O
for f in 0 1; do
  HIPDSML_PK_OWNLAST=$f timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 2,8 --stamps $O/st_$f.jsonl > /dev/null 2>$O/err_$f.txt
done
for k in 1 2 3; do
  for f in 0 1; do
    HIPDSML_PK_OWNLAST=$f timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 2,4,8 2>/dev/null | cut -c1-100 | sed "s/^/ownlast=$f probe /"
  done
done
