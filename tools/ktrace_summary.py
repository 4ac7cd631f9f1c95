"""Per-kernel launch statistics from a rocprofv3 kernel trace (run_kernel_trace.csv),
with each kernel's first `--skip` launches (warm-up) left out.

rocprofv3 --stats averages every launch, warm-up included; this reads the
per-dispatch trace of the same run instead. Usage:
  ktrace_summary.py <kernel_trace.csv> [--skip N] [--match REGEX] [--json OUT]
"""
import argparse
import csv
import json
import re
import statistics
import sys


def summarize(path, skip=0, match=None):
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if match and not re.search(match, name):
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", "")))
    rows.sort()
    by = {}
    for s, e, name, q in rows:
        by.setdefault(name, []).append((e - s) / 1e6)
    out = {}
    for name, ms in by.items():
        kept = ms[skip:] if len(ms) > skip else []
        if not kept:
            continue
        out[name] = {"launches": len(ms), "skipped": len(ms) - len(kept), "calls": len(kept),
                     "avg_ms": round(statistics.mean(kept), 4), "median_ms": round(statistics.median(kept), 4),
                     "min_ms": round(min(kept), 4), "max_ms": round(max(kept), 4)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=0, help="launches of each kernel left out (warm-up)")
    ap.add_argument("--match", default=None, help="only kernels whose name matches")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = summarize(a.trace, a.skip, a.match)
    text = json.dumps(out, indent=1, sort_keys=True)
    if a.json:
        with open(a.json, "w") as f:
            f.write(text + "\n")
    sys.stdout.write(text + "\n")


if __name__ == "__main__":
    main()
