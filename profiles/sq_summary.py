#!/usr/bin/env python
"""Sum SQ counters over all launches of one kernel from pmc_sq.sh's passes."""
import csv
import glob
import os
import sys
from collections import defaultdict

out, kern = sys.argv[1], sys.argv[2]
tot = defaultdict(float)
n = defaultdict(int)
for path in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            if kern in row["Kernel_Name"]:
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
                n[row["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:18.4g}  (records {n[k]})")
w = tot.get("SQ_WAVE_CYCLES", 0)
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_LDS", "SQ_INST_CYCLES_VMEM"):
        if k in tot:
            print(f"{k:28s} / WAVE_CYCLES = {tot[k] / w:.3f}")
