"""Per-kernel launch durations of a bench's full-size steps from a rocprofv3
kernel_trace.csv: for each kernel, the launches of at least half its longest
(the parity checks on the 1x base file are far shorter), their count, median
and min in ms. A kernel_stats.csv averages every launch together, which for
the codec benches mixes the full-size steps with those checks.
Usage: ktrace_steps.py <trace dir or csv>... -> JSON on stdout."""
import csv
import glob
import json
import os
import re
import statistics
import sys

out = {}
for arg in sys.argv[1:]:
    paths = [arg] if arg.endswith(".csv") else glob.glob(os.path.join(arg, "**", "*kernel_trace.csv"), recursive=True)
    durs = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
            durs.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    res = {}
    for name, ds in durs.items():
        big = [d for d in ds if d >= 0.5 * max(ds)]
        res[name] = {"launches": len(big), "median_ms": round(statistics.median(big), 4), "min_ms": round(min(big), 4),
                     "all_launches": len(ds)}
    out[arg] = dict(sorted(res.items(), key=lambda kv: -kv[1]["median_ms"]))
json.dump(out, sys.stdout, indent=1)
print()
