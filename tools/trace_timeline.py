"""Timeline of one sample() call from a rocprofv3 kernel trace (tools/gpu_trace.sh).

usage: python tools/trace_timeline.py kt_kernel_trace.csv [call index]
Calls are split at the std-euclid filter's bitonic sort (first kernel of a sample() call).
Prints per queue: busy time, and the main queue's idle gaps > 0.2 ms with what ran meanwhile.
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
want = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
starts = [i for i, r in enumerate(rows) if "k_bitonic_step" in r["Kernel_Name"] and
          (i == 0 or "k_bitonic_step" not in rows[i - 1]["Kernel_Name"])]
print(f"{len(starts)} calls")
a = starts[want]
b = starts[want + 1] if want + 1 < len(starts) else len(rows)
call = rows[a:b]
t0 = call[0]["s"]
t1 = max(r["e"] for r in call)
print(f"call {want}: {len(call)} dispatches, {(t1 - t0) / 1e6:.2f} ms")
byq = defaultdict(list)
for r in call:
    byq[r["Queue_Id"]].append(r)


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("npfn::", "")[:48]


for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
    busy = sum(r["e"] - r["s"] for r in rs)
    kinds = defaultdict(float)
    for r in rs:
        kinds[short(r["Kernel_Name"])] += (r["e"] - r["s"]) / 1e6
    top = sorted(kinds.items(), key=lambda kv: -kv[1])[:6]
    print(f"queue {q}: {len(rs)} dispatches, busy {busy / 1e6:.2f} ms, span {(rs[0]['s'] - t0) / 1e6:.2f}.."
          f"{(rs[-1]['e'] - t0) / 1e6:.2f} ms; " + ", ".join(f"{k} {v:.2f}" for k, v in top))
main = max(byq.items(), key=lambda kv: len(kv[1]))[1]
print("main-queue gaps > 0.2 ms:")
tot = 0.0
for p, n in zip(main, main[1:]):
    g = n["s"] - p["e"]
    if g > 200_000:
        tot += g
        other = [short(r["Kernel_Name"]) for r in call if r["s"] < n["s"] and r["e"] > p["e"] and r not in main]
        print(f"  {(p['e'] - t0) / 1e6:8.2f} ms +{g / 1e6:6.2f} ms after {short(p['Kernel_Name'])} -> "
              f"{short(n['Kernel_Name'])}; meanwhile {sorted(set(other))[:4]}")
print(f"total main gaps > 0.2 ms: {tot / 1e6:.2f} ms")
