"""Timeline of one end-to-end scan from a rocprofv3 --kernel-trace
--memory-copy-trace run of tools/bench_e2e.py --reps 1 (the timed scan): the
rio kernels and the SDMA copies, ms from the timed scan's first copy, as the
JSON under profiles/ (r06_e2e_*_trace_summary.json). The timed scan is the
last one: its first copy is the last H2D copy that follows a gap of more than
`--gap` ms with no copy or rio kernel.

  python tools/e2e_timeline.py gpurun_out/r06_e2e_trace_c3 [--gap 50] > profiles/...json
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gap", type=float, default=50.0)
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    ev = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if k.startswith("rio::"):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    for f in glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = r.get("Direction", "") or r.get("Operation", "")
            n = int(r.get("Bytes", 0) or 0) if (r.get("Bytes") or "").isdigit() else None
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + d + ("" if n is None else " %d B" % n)))
    ev.sort()
    start = 0
    for i in range(1, len(ev)):
        if (ev[i][0] - max(e[1] for e in ev[:i])) / 1e6 > a.gap:
            start = i
    ev = ev[start:]
    t0 = ev[0][0]
    out = {"source": a.source or "rocprofv3 --kernel-trace --memory-copy-trace of tools/bench_e2e.py --reps 1; ms from the timed scan's first event",
           "events": [{"start_ms": round((s - t0) / 1e6, 3), "end_ms": round((e - t0) / 1e6, 3), "what": w} for s, e, w in ev
                      if w.startswith("COPY") or (e - s) > 200000]}
    print(json.dumps(out, indent=0))


if __name__ == "__main__":
    main()
