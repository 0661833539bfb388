"""Compare rocprofv3 kernel-stats CSVs of several runs: per kernel, calls and average / total time.

usage: python tools/kstats_cmp.py DIR_OR_CSV[=label] ... [--grep PATTERN]"""
import csv
import glob
import json
import os
import re
import sys


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_stats.csv"), recursive=True)[0]
    return {r["Name"]: r for r in csv.DictReader(open(path))}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--grep")]
    pat = None
    for a in sys.argv[1:]:
        if a.startswith("--grep="):
            pat = re.compile(a.split("=", 1)[1])
    runs = []
    for a in args:
        path, _, label = a.partition("=")
        runs.append((label or os.path.basename(path.rstrip("/")), load(path)))
    names = sorted({n for _, r in runs for n in r}, key=lambda n: -float(runs[0][1].get(n, {}).get("TotalDurationNs", 0)))
    print(f"{'kernel':60s}" + "".join(f"{lab:>28s}" for lab, _ in runs))
    for n in names:
        if pat and not pat.search(n):
            continue
        cells = []
        for _, r in runs:
            e = r.get(n)
            cells.append(f"{int(e['Calls']):6d} x {float(e['AverageNs']) / 1e3:8.1f} us {float(e['TotalDurationNs']) / 1e6:7.2f} ms"
                         if e else f"{'-':>28s}")
        print(f"{n[:60]:60s}" + "".join(f"{c:>28s}" for c in cells))


if __name__ == "__main__":
    main()
