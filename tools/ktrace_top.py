"""Per-launch durations (ms) of the long kernels in a rocprofv3 kernel_trace.csv."""
import collections
import csv
import sys

for path in sys.argv[1:]:
    big = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        big[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    print(path)
    for k, v in big.items():
        if max(v) > 1:
            print("  %-44s %s" % (k[:44], " ".join("%.1f" % x for x in v[-5:])))
