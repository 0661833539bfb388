"""Print the headline and per-kernel summary of one bench.py JSON line (tools/gpu.sh quick)."""
import json
import sys

d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"value {d['value']:.1f} {d['unit']}  ms/step {d['ms_per_step']:.2f}  roofline {d.get('roofline', {}).get('frac')}")
for k, v in (d.get("kernels") or {}).items():
    print(f"  {k:28s} " + "  ".join(f"{a}={v[a]}" for a in ("ms_per_step", "launches", "tflops", "gbs", "fallback_frac") if a in v))
