"""Average per-dispatch PMC values per kernel from rocprofv3 counter_collection CSVs.

FETCH_SIZE / WRITE_SIZE are in KB (1024 B). On gfx950 FETCH_SIZE reports half
the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM section):
`fetch_bytes` is the doubled value, `fetch_bytes_raw` the counter as read.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows.extend(csv.DictReader(fh))
    return rows


def main(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for r in load(d):
            name = r.get("Kernel_Name", "")
            short = name.split("(")[0].replace("void ", "").strip()
            acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, ctrs in acc.items():
        e = {"dispatches": max(len(v) for v in ctrs.values())}
        if "FETCH_SIZE" in ctrs:
            v = ctrs["FETCH_SIZE"]
            e["fetch_bytes_raw"] = sum(v) / len(v) * 1024
            e["fetch_bytes"] = 2 * e["fetch_bytes_raw"]
        if "WRITE_SIZE" in ctrs:
            v = ctrs["WRITE_SIZE"]
            e["write_bytes"] = sum(v) / len(v) * 1024
        for c, v in ctrs.items():  # other counters: mean per dispatch
            if c not in ("FETCH_SIZE", "WRITE_SIZE"):
                e[c] = sum(v) / len(v)
        out[k] = e
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1:])
