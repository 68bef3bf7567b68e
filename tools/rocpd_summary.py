#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (ROCm 7 default output): per-kernel
calls / total / avg / min / max (ns) and the mean gap between consecutive
dispatches on the same queue.  Usage: rocpd_summary.py run_results.db [--csv out]"""
import argparse
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default="")
    ap.add_argument("--skip", type=int, default=0, help="ignore the first N dispatches (warm-up)")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    q = f"select {name_col}, start, end, queue_id from kernels order by start"
    try:
        rows = list(db.execute(q))
    except sqlite3.OperationalError:
        rows = list(db.execute(f"select {name_col}, start, end, 0 from kernels order by start"))
    rows = rows[a.skip:]
    agg = defaultdict(list)
    for name, s, e, _ in rows:
        agg[name].append(e - s)
    total = sum(sum(v) for v in agg.values())
    out = []
    for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append({"name": name[:140], "calls": len(d), "total_ns": sum(d),
                    "avg_ns": round(sum(d) / len(d), 1), "median_ns": statistics.median(d),
                    "min_ns": min(d), "max_ns": max(d), "pct": round(100 * sum(d) / total, 2)})
    byq = defaultdict(list)
    for name, s, e, qid in rows:
        byq[qid].append((s, e))
    gaps = []
    for v in byq.values():
        for (s0, e0), (s1, e1) in zip(v, v[1:]):
            if s1 >= e0:
                gaps.append(s1 - e0)
    span = (rows[-1][2] - rows[0][1]) if rows else 0
    w = csv.DictWriter(sys.stdout, fieldnames=list(out[0].keys())) if out else None
    if w:
        w.writeheader()
        w.writerows(out)
    print(f"# dispatches={len(rows)} busy_ns={total} span_ns={span} "
          f"median_gap_ns={statistics.median(gaps) if gaps else 0}")
    if a.csv and out:
        with open(a.csv, "w", newline="") as fh:
            cw = csv.DictWriter(fh, fieldnames=list(out[0].keys()))
            cw.writeheader()
            cw.writerows(out)
            fh.write(f"# dispatches={len(rows)} busy_ns={total} span_ns={span} "
                     f"median_gap_ns={statistics.median(gaps) if gaps else 0}\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
