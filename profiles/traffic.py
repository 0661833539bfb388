#!/usr/bin/env python
"""Per-launch HBM traffic of one kernel from rocprofv3 --pmc passes.

Reads the FETCH_SIZE and WRITE_SIZE counter_collection CSVs (separate passes)
and applies the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE
reports half the bytes of a wide (16 B/lane) coalesced read, so it is doubled;
WRITE_SIZE is taken as is.  Counters are in KiB.  Output: traffic.json with the
mean bytes per launch (the same per-launch averaging as bench.py's roofline).

usage: traffic.py FETCH.csv WRITE.csv KERNEL_SUBSTRING OUT.json [SOURCE_LABEL]
SOURCE_LABEL (e.g. "profiles/r05/pmc_*_r05x, tree <commit>") is stored as "source" and shows up as
the bench line's roofline.traffic_source.
"""
import csv
import json
import sys


def per_launch(path, kernel):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fetch_csv, write_csv, kernel, out = sys.argv[1:5]
    label = sys.argv[5] if len(sys.argv) > 5 else f"{fetch_csv} + {write_csv}"
    fk = per_launch(fetch_csv, kernel)
    wk = per_launch(write_csv, kernel)
    fetch = sum(fk) / len(fk) * 1024 * 2.0
    write = sum(wk) / len(wk) * 1024
    res = {"kernel": kernel, "bytes_per_launch": fetch + write, "fetch_bytes_per_launch": fetch,
           "write_bytes_per_launch": write, "launches_fetch_pass": len(fk), "launches_write_pass": len(wk),
           "correction": "FETCH_SIZE x2 (gfx950 wide-read under-count), KiB -> bytes", "source": label}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
