"""Host issue time vs GPU start time of one sample() call (tools/gpu_trace_api.sh output).

usage: python tools/trace_api.py <dir with kt_kernel_trace.csv, kt_hip_api_trace.csv> [call index]
For every main-queue idle gap > 0.2 ms: when the host issued the dispatch that ended the gap
(the launch call's timestamp) -- a late issue means the host, not a stream dependency, held it
back -- and the host API calls that took > 0.2 ms during the call.
"""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1]
want = int(sys.argv[2]) if len(sys.argv) > 2 else 2


def load(name):
    p = [os.path.join(d, f) for f in os.listdir(d) if f.endswith(name)]
    return list(csv.DictReader(open(p[0]))) if p else []


kt = load("kernel_trace.csv")
api = load("hip_api_trace.csv")
for r in kt + api:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
kt.sort(key=lambda r: r["s"])
by_corr = {r["Correlation_Id"]: r for r in api}
starts = [i for i, r in enumerate(kt) if "k_bitonic_step" in r["Kernel_Name"] and
          (i == 0 or "k_bitonic_step" not in kt[i - 1]["Kernel_Name"])]
a = starts[want]
b = starts[want + 1] if want + 1 < len(starts) else len(kt)
call = kt[a:b]
t0, t1 = call[0]["s"], max(r["e"] for r in call)
print(f"{len(starts)} calls; call {want}: {len(call)} dispatches, {(t1 - t0) / 1e6:.2f} ms")
byq = defaultdict(list)
for r in call:
    byq[r["Queue_Id"]].append(r)
main = max(byq.values(), key=len)


def short(n):
    return n.split("(")[0].replace("void ", "").replace("npfn::", "")[:40]


def issued(r):
    c = by_corr.get(r["Correlation_Id"])
    return (c["s"] - t0) / 1e6 if c else float("nan")


print("main-queue gaps > 0.2 ms (t = ms from call start):")
for p, n in zip(main, main[1:]):
    g = n["s"] - p["e"]
    if g > 200_000:
        print(f"  prev {short(p['Kernel_Name'])} ends {(p['e'] - t0) / 1e6:7.2f}; next {short(n['Kernel_Name'])} "
              f"issued {issued(n):7.2f}, starts {(n['s'] - t0) / 1e6:7.2f} (+{g / 1e6:.2f})")
tid = defaultdict(int)
for r in api:
    if t0 <= r["s"] <= t1:
        tid[r["Thread_Id"]] += 1
print("host threads issuing during the call:", dict(tid))
print("host API calls > 0.2 ms during the call:")
for r in sorted(api, key=lambda r: r["s"]):
    if t0 <= r["s"] <= t1 and r["e"] - r["s"] > 200_000:
        print(f"  {(r['s'] - t0) / 1e6:7.2f} +{(r['e'] - r['s']) / 1e6:6.2f} ms {r['Function']} (thread {r['Thread_Id']})")
# the host's issue rate: launches per ms over the call
la = sorted(r["s"] for r in api if t0 <= r["s"] <= t1 and "Launch" in r["Function"])
if la:
    print(f"launch calls: {len(la)}, first {(la[0] - t0) / 1e6:.2f} ms, last {(la[-1] - t0) / 1e6:.2f} ms")
