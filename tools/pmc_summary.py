"""Summarise rocprofv3 --pmc CSV passes: per counter, the mean value per
dispatch of the kernel (name substring) with the most dispatches.
usage: pmc_summary.py OUT.json name=substring:dir[,dir...] ..."""
import collections
import csv
import glob
import json
import os
import sys


def load(dirs, sub):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "")
                    if sub in k:
                        vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not vals:
        return {"error": f"no kernel matching {sub!r}"}
    k = max(vals, key=lambda x: max(len(v) for v in vals[x].values()))
    out = {c: round(sum(v) / len(v), 1) for c, v in sorted(vals[k].items())}
    out["kernel"] = k[:100]
    return out


res = {}
for arg in sys.argv[2:]:
    name, spec = arg.split("=", 1)
    sub, dirs = spec.split(":", 1)
    res[name] = load(dirs.split(","), sub)
json.dump(res, open(sys.argv[1], "w"), indent=1)
print(json.dumps(res, indent=1))
