"""Instruction budget of one kernel from its device assembly: dynamic counts per opcode class,
loop bodies weighted by their trip counts (given on the command line, innermost first).

usage: python tools/isa_budget.py KERNEL.s SYMBOL_PREFIX [trip ...]
Classes: mfma, exp/transcendental, bf16 pack, fma/mul/add (f32 math), max/min, cndmask/select,
int/address math, mov, permlane/dpp/shuffle, ds (LDS), global/buffer (VMEM), salu, waitcnt, nop,
barrier."""
import re
import sys
from collections import Counter

path, sym = sys.argv[1], sys.argv[2]
trips = [int(t) for t in sys.argv[3:]]
lines = open(path).read().split("\n")
st = next(i for i, l in enumerate(lines) if l.startswith(sym) and ":" in l.split(";")[0])
en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith("s_endpgm"))
body = lines[st:en + 1]


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_", op):
        return "transcendental"
    if op.startswith("v_cvt_pk_bf16") or op.startswith("v_perm_b32") or op.startswith("v_pack"):
        return "bf16 pack"
    if re.match(r"v_(pk_)?(fma|fmac|mul|add|sub|subrev|mac)_f(32|64)", op) or op.startswith("v_pk_fma") \
            or op.startswith("v_pk_mul") or op.startswith("v_pk_add"):
        return "f32 math"
    if re.match(r"v_(max|min|max3|min3|med3)_", op):
        return "max/min"
    if op.startswith("v_cndmask") or op.startswith("v_cmp"):
        return "cmp/select"
    if op.startswith("v_mov") or op.startswith("v_accvgpr"):
        return "mov"
    if "permlane" in op or "dpp" in op or op.startswith("v_readlane") or op.startswith("v_readfirstlane") \
            or op.startswith("v_writelane") or op.startswith("ds_swizzle") or op.startswith("ds_bpermute"):
        return "cross-lane"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_") or op.startswith("scratch_"):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "int/other valu"
    return None


ops = []
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = len(ops)
        continue
    t = l.strip()
    if not t or t.startswith(";") or t.startswith("."):
        continue
    op = t.split()[0]
    ops.append(op if not op.endswith(":") else None)
    tgt = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", t)
    if tgt:
        ops[-1] = (op, tgt.group(1) or tgt.group(2))
# loops = backward branches
weight = [1] * len(ops)
loops = []
for i, o in enumerate(ops):
    if isinstance(o, tuple) and o[1] in labels and labels[o[1]] <= i:
        loops.append((labels[o[1]], i))
loops = sorted(set(loops), key=lambda r: r[1] - r[0])
for k, (a, b) in enumerate(loops):
    t = trips[k] if k < len(trips) else 1
    for i in range(a, b + 1):
        weight[i] *= t
cnt = Counter()
for o, w in zip(ops, weight):
    if o is None:
        continue
    op = o[0] if isinstance(o, tuple) else o
    c = klass(op)
    if c:
        cnt[c] += w
print(f"{sym}: {len(loops)} loops {[(b - a) for a, b in loops]} trips {trips}")
mf = cnt["mfma"] or 1
valu = sum(v for k, v in cnt.items() if k in ("transcendental", "bf16 pack", "f32 math", "max/min", "cmp/select",
                                               "mov", "int/other valu", "cross-lane"))
for k, v in cnt.most_common():
    print(f"  {k:16s} {v:8d}  {v / mf:6.2f} per MFMA")
print(f"  VALU total       {valu:8d}  {valu / mf:6.2f} per MFMA")
