set -e
mkdir -p gpurun_out/pkh
for h in 0 1 2 3; do
  timeout -k 10 120 python tools/pk_probe.py --algo 4 --ranks 8 --helpers $h --stamps gpurun_out/pkh/p_$h.jsonl 2>/dev/null | cut -c1-110
  timeout -k 10 120 python tools/pk_probe.py --algo 4 --ranks 8 --helpers $h --mirror 2>/dev/null | cut -c1-110
done
