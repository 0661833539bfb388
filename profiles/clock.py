#!/usr/bin/env python
"""Effective shader clock per kernel from a rocprofv3 GRBM_GUI_ACTIVE pass (MI355X_MICROARCH.md
'DVFS give-back': clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time; reliable on dispatches of
a few ms, reads high below ~0.3 ms).  Durations come from the counter CSV's timestamps or, when
absent, from the same pass's kernel trace (joined on Dispatch_Id).

usage: clock.py COUNTER.csv [KERNEL_TRACE.csv] [regex]
"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def main():
    pmc = list(csv.DictReader(open(sys.argv[1])))
    trace = {}
    if len(sys.argv) > 2 and sys.argv[2].endswith(".csv"):
        for r in csv.DictReader(open(sys.argv[2])):
            trace[r["Dispatch_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    rx = re.compile(sys.argv[3] if len(sys.argv) > 3 else ".")
    per = defaultdict(list)
    for r in pmc:
        if r["Counter_Name"] != "GRBM_GUI_ACTIVE" or not rx.search(r["Kernel_Name"]):
            continue
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        elif r["Dispatch_Id"] in trace:
            t0, t1 = trace[r["Dispatch_Id"]]
        else:
            continue
        dur = (t1 - t0) * 1e-9
        if dur < 1e-3:  # the quotient reads high on short dispatches
            continue
        name = re.sub(r"\(.*", "", r["Kernel_Name"])[:60]
        per[name].append(float(r["Counter_Value"]) / 8.0 / dur / 1e9)
    for name, v in sorted(per.items(), key=lambda kv: -len(kv[1])):
        print(f"{name:60s} dispatches {len(v):5d}  clock GHz median {statistics.median(v):.3f}  "
              f"min {min(v):.3f}  max {max(v):.3f}")


if __name__ == "__main__":
    main()
