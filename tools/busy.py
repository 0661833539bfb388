"""GPU busy time of a rocprofv3 kernel trace, per call: the union of all kernels' [start, end)
intervals (any queue / stream) against the call's span, and the largest idle gaps with the kernels
either side -- what of a call's wall clock no kernel covers (host syncs, launch gaps).

usage: python tools/busy.py KERNEL_TRACE.csv [call-start regex, default k_fill] [gaps to list]
A call spans from one match of the regex to the next (the last call: to the trace's end).
"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    rx = re.compile(sys.argv[2] if len(sys.argv) > 2 else "k_fill")
    ngap = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-48:]) for r in rows]
    marks = [i for i, k in enumerate(ks) if rx.search(k[2])]
    for c, i0 in enumerate(marks):
        i1 = marks[c + 1] if c + 1 < len(marks) else len(ks)
        seg = ks[i0:i1]
        t0, t1 = seg[0][0], max(k[1] for k in seg)
        busy, cur_s, cur_e, gaps = 0, seg[0][0], seg[0][1], []
        prev = seg[0][2]
        for s, e, n in seg[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, prev, n))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            if e >= cur_e:
                prev = n
        busy += cur_e - cur_s
        span = t1 - t0
        gaps.sort(reverse=True)
        print(f"call {c}: span {span / 1e6:8.2f} ms  busy {busy / 1e6:8.2f} ms ({busy / span:6.1%})  "
              f"idle {(span - busy) / 1e6:6.2f} ms in {len(gaps)} gaps")
        for g, a, b in gaps[:ngap]:
            print(f"    {g / 1e3:8.1f} us  after {a}  before {b}")


if __name__ == "__main__":
    main()
