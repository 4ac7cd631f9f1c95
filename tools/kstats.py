"""Print a rocprofv3 kernel_stats.csv compactly: name (shortened), calls, total ms, avg us."""
import csv
import re
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        rows = list(csv.DictReader(f))
    print(path)
    for r in rows[:int(12)]:
        name = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")
        print("  %-40s %6s calls %10.3f ms  avg %10.1f us  %5.1f%%" % (
            name[:40], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e3,
            float(r["Percentage"])))
