"""Sum rocprofv3 --pmc counter_collection.csv rows per kernel: kernel -> counter -> (sum over
dispatches), plus dispatch count. Usage: pmc_sum.py <dir>... [--match substr]"""
import collections
import csv
import glob
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = None
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args = [a for a in args if a != match]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in args:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
            if match and match not in k:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
for k in sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", 0)):
    print(k, "dispatches", len(disp[k]))
    for c, v in sorted(tot[k].items()):
        print("   %-24s %16.0f" % (c, v))
