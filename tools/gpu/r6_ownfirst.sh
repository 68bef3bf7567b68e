# pkx layer-1 dZ1 poll: own rows first (HIPDSML_PK_OWN_FIRST 1) vs merged (0),
# lone-replica probe and mirror mode at N = 2 / 4 / 8, alternating; then the
# replay test with the winner's setting exercised through both values
set -e
O=gpurun_out/${1:-r6own}
mkdir -p $O
for k in 1 2; do
  for f in 0 1; do
    HIPDSML_PK_OWN_FIRST=$f timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 2,4,8 2>/dev/null | cut -c1-100 | sed "s/^/own_first=$f probe /"
    HIPDSML_PK_OWN_FIRST=$f timeout -k 10 150 python tools/pk_probe.py --algo 4 --ranks 4,8 --mirror 2>/dev/null | cut -c1-100 | sed "s/^/own_first=$f mirror /"
  done
done
