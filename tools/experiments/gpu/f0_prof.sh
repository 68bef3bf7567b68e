set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_f0 -o run -- python3 $R/tools/f0_variants.py > $R/gpurun_out/prof_f0.log 2>&1
cd $R && python - <<'PY'
import csv, glob, statistics
f = glob.glob("gpurun_out/prof_f0/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "rows64" in r["Kernel_Name"] or "skinny" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
for i, n in enumerate(["rows64", "skinny_s1", "skinny_s2", "skinny_s3", "skinny_s4"]):
    seg = d[30 * i + 5: 30 * i + 30]
    print(n, round(statistics.median(seg), 2))
PY
