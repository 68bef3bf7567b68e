# Head kernel variants under a kernel trace (durations per variant, in call order).
set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_head -o run -- python3 $R/tools/head_bench.py > $R/gpurun_out/prof_head.log 2>&1
cd $R && python - <<'PY'
import csv, glob, statistics
f = glob.glob("gpurun_out/prof_head/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "head_softmax" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
names = ["full", "no_dzp", "no_logits_no_dzp", "dbg1_no_atomics", "dbg2_no_dzp", "dbg3_neither", "stamped"]
i = 0
for n in names:
    seg = d[i:i + 55] if n != "stamped" else d[i:i + 1]
    i += len(seg)
    if seg:
        print(n, round(statistics.median(seg), 2), "us over", len(seg))
PY
